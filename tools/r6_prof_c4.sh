#!/bin/bash
# per-step kernel summaries of the C4 step, fp8 and bf16 (rocprofv3 kernel trace)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r6}
export TMPDIR=/tmp
for p in ${PRECS:-fp8 bf16}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4${p}_${TAG} -o run --output-format csv -- \
    python bench.py --config c4 --precision $p --no-cpu-baseline --no-parity --no-u8-leg --no-kernel-timer --steps 8 \
    > gpurun_out/prof_c4${p}_${TAG}.log 2>&1 || { tail -30 gpurun_out/prof_c4${p}_${TAG}.log; exit 1; }
  f=$(find gpurun_out/prof_c4${p}_${TAG} -name "*kernel_trace.csv" | head -1)
  python tools/step_kernels.py "$f" 3 45 > gpurun_out/c4_${p}_${TAG}_step_kernels.txt || exit 1
  rm -f "$f"
  head -40 gpurun_out/c4_${p}_${TAG}_step_kernels.txt
done
