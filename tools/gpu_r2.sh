#!/bin/bash
# One gpurun call: GPU tests (all, not stopping at assertion failures), then a
# short bench without the CPU baseline. Each GPU step has its own limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-r2}"
SEL="${SEL:-tests}"
timeout -k 10 ${PYT_LIMIT:-600} python -u -m pytest $SEL -v -m gpu --timeout 150 --timeout-method thread ${PYTEST_ARGS} \
  > gpurun_out/pytest_${TAG}.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_${TAG}.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
exit $rc
