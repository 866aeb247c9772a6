#!/bin/bash
# Aux-ring depth of the mul-aux epilogue (GEMM4_EPI_PF_AUX): default build vs
# libmaeclip_pfa3.so -- GEMM tests on both, per-launch epilogue cost, whole-step A/B.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r5aa}
for L in libmaeclip.so libmaeclip_pfa3.so; do
  MAECLIP_LIB=mae_clip_amd/$L timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_kernels_gpu.py -k "gemm" > gpurun_out/pfa_tests_${L}_$T.txt 2>&1 || { tail -30 gpurun_out/pfa_tests_${L}_$T.txt; exit 1; }
  tail -1 gpurun_out/pfa_tests_${L}_$T.txt
  MAECLIP_LIB=mae_clip_amd/$L timeout -k 10 300 python -u tools/epi_cost_probe.py 2>&1 | sed "s/^/$L /" >> gpurun_out/pfa_epi_$T.txt || exit 1
done
ROUNDS=2 bash tools/env_ab.sh "-" "MAECLIP_LIB=mae_clip_amd/libmaeclip_pfa3.so" > gpurun_out/pfa_step_$T.txt 2>&1 || exit 1
cat gpurun_out/pfa_step_$T.txt
