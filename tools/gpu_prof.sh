#!/bin/bash
# pytest -m gpu, bench (no CPU baseline), rocprofv3 kernel-trace stats of a short bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-prof}"
if [ -z "$NO_TESTS" ]; then
  TAG=$TAG NO_BENCH=1 PYT_LIMIT=600 bash tools/gpu_r2.sh; rc=$?
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
cat gpurun_out/bench_${TAG}.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity --no-kernel-timer ${BENCH_ARGS} > gpurun_out/prof_${TAG}.log 2>&1 || { tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 13 | head -45
