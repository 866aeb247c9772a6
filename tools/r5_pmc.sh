#!/bin/bash
# Round-5 evidence pass (one call): per-step kernel summary of the default C2
# bench, in-step PMC traffic of the decoder's grouped weight-gradient launch
# (PICK 0/2: the decoder launch of each step), standalone PMC traffic of the
# dominant forward / dgrad shape (enc fc2 fwd + residual, M 6400 N 768 K 3072).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG} -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-parity --steps 20 > gpurun_out/prof_${TAG}.log 2>&1 || { tail -30 gpurun_out/prof_${TAG}.log; exit 1; }
f=$(find gpurun_out/prof_${TAG} -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py "$f" 5 60 > gpurun_out/step_kernels_${TAG}.txt || exit 1
head -14 gpurun_out/step_kernels_${TAG}.txt
TAG=${TAG}_wgdec PICK=0/2 timeout -k 10 900 bash tools/pmc_instep.sh wgrad4_kernel 131072 "wgrad_grouped M50432 x32 N512 K2048 bf16>f32" > gpurun_out/pmcstep_${TAG}.txt 2>&1 || { tail -20 gpurun_out/pmcstep_${TAG}.txt; exit 1; }
tail -1 gpurun_out/pmcstep_${TAG}.txt
TAG=${TAG}_encfc2 timeout -k 10 400 bash tools/pmc_traffic.sh 6400 768 3072 0 0 2 > gpurun_out/pmc_${TAG}.txt 2>&1 || { tail -20 gpurun_out/pmc_${TAG}.txt; exit 1; }
tail -1 gpurun_out/pmc_${TAG}.txt
