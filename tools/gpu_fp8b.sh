#!/bin/bash
# fp8 tests, C4 fp8 bench, rocprof kernel stats of the C4 fp8 step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fp8_gpu.py -q -s -m gpu --timeout 200 --timeout-method thread > gpurun_out/pt_fp8.log 2>&1
rc=$?
grep -E "FAIL|fp8 loss|worst|Error|assert|passed|failed" gpurun_out/pt_fp8.log | head -30
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-parity --config c4 --precision fp8 > gpurun_out/bench_c4_fp8.json 2> gpurun_out/bench_c4_fp8.err || { tail -30 gpurun_out/bench_c4_fp8.err; exit 1; }
cat gpurun_out/bench_c4_fp8.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4f8 -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-parity --no-kernel-timer --config c4 --precision fp8 > gpurun_out/prof_c4f8.log 2>&1 || { tail -30 gpurun_out/prof_c4f8.log; exit 1; }
f=$(find gpurun_out/prof_c4f8 -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 8 30
exit $rc
