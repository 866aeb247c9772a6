#!/bin/bash
# fp8 kernel/model tests, then C1 / C4 (bf16, fp8) bench lines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -v -s -m gpu --timeout 200 --timeout-method thread > gpurun_out/pt_fp8.log 2>&1
rc=$?
grep -E "PASS|FAIL|ERROR|fp8 loss|worst|Error|assert" gpurun_out/pt_fp8.log | head -60
tail -3 gpurun_out/pt_fp8.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for a in "c1 bf16" "c4 bf16" "c4 fp8"; do
  set -- $a
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-parity --config $1 --precision $2 > gpurun_out/bench_$1_$2.json 2> gpurun_out/bench_$1_$2.err || { tail -30 gpurun_out/bench_$1_$2.err; exit 1; }
  cat gpurun_out/bench_$1_$2.json
done
exit $rc
