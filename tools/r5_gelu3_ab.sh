#!/bin/bash
# Stage-wise GELU epilogue (gelu_pairs) vs the pair-by-pair form (libmaeclip_oldgelu.so):
# GEMM tests on the new build, per-launch epilogue cost on both, whole-step A/B.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r5z}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm" \
  tests/test_fp8_gpu.py > gpurun_out/gelu3_tests_$T.txt 2>&1 || { tail -30 gpurun_out/gelu3_tests_$T.txt; exit 1; }
tail -2 gpurun_out/gelu3_tests_$T.txt
for L in libmaeclip.so libmaeclip_oldgelu.so; do
  MAECLIP_LIB=mae_clip_amd/$L timeout -k 10 300 python -u tools/epi_cost_probe.py 2>&1 | sed "s/^/$L /" >> gpurun_out/gelu3_epi_$T.txt || exit 1
done
ROUNDS=2 bash tools/env_ab.sh "-" "MAECLIP_LIB=mae_clip_amd/libmaeclip_oldgelu.so" > gpurun_out/gelu3_step_$T.txt 2>&1 || exit 1
cat gpurun_out/gelu3_step_$T.txt
