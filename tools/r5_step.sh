#!/bin/bash
# this round's step-level probe: per-step kernel summary of the default build,
# then whole-step A/B of GEMM settings on the same box
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r5}
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-parity --steps 20 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py "$f" 5 40 > gpurun_out/step_kernels_${TAG}.txt || exit 1
head -12 gpurun_out/step_kernels_${TAG}.txt
ROUNDS=2 timeout -k 10 900 bash tools/env_ab.sh "$@" > gpurun_out/envab_${TAG}.txt 2>&1 || { cat gpurun_out/envab_${TAG}.txt; exit 1; }
cat gpurun_out/envab_${TAG}.txt
