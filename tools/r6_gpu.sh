#!/bin/bash
# Round-6 GPU pass: the GPU test suite (parity records to gpurun_out/), then
# optional extra steps named on the command line:
#   curve   tools/curve_diag.py (C0 fp32 curve: which step / op leaves fp64)
#   bench   default bench.py line (C2) into gpurun_out/bench_${TAG}.json
#   prof    rocprofv3 kernel-trace summary of the C2 step
#   c4      C4 bf16 / fp8 bench lines (tools/cfg_runs.sh)
#   notests skip the test suite
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r6}
export TMPDIR=/tmp
export MAECLIP_PARITY_OUT=$PWD/gpurun_out/parity_${TAG}.jsonl
want() { for a in "${@:2}"; do [ "$a" = "$1" ] && return 0; done; return 1; }
if ! want notests "$@"; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_${TAG}.txt 2>&1 || { tail -40 gpurun_out/gpu_tests_${TAG}.txt; exit 1; }
  tail -3 gpurun_out/gpu_tests_${TAG}.txt
fi
if want curve "$@"; then
  timeout -k 10 300 python -u tools/curve_diag.py --out gpurun_out/curve_diag_${TAG}.json \
    > gpurun_out/curve_diag_${TAG}.txt 2>&1 || { tail -30 gpurun_out/curve_diag_${TAG}.txt; exit 1; }
  cat gpurun_out/curve_diag_${TAG}.txt
fi
if want bench "$@"; then
  timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err \
    || { tail -30 gpurun_out/bench_${TAG}.err; exit 1; }
  cat gpurun_out/bench_${TAG}.json
fi
if want prof "$@"; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-parity --steps 20 > gpurun_out/prof_${TAG}.log 2>&1 \
    || { tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
  f=$(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
  python tools/step_kernels.py "$f" 5 40 > gpurun_out/step_kernels_${TAG}.txt || exit 1
  head -14 gpurun_out/step_kernels_${TAG}.txt
fi
if want c4 "$@"; then
  timeout -k 10 900 bash tools/cfg_runs.sh > gpurun_out/cfgs_${TAG}.txt 2>&1 || { tail -30 gpurun_out/cfgs_${TAG}.txt; exit 1; }
  cat gpurun_out/cfgs_${TAG}.txt
fi
exit 0
