#!/bin/bash
# packed-f32 GELU / GELU' epilogue (gelu_pair2) vs the scalar one: GEMM tests,
# epilogue shapes alone, whole step (same box)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r5}
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "gemm or gelu or epilog or model" --timeout 120 --timeout-method thread > gpurun_out/pytest_gelu_$T.log 2>&1 || { tail -30 gpurun_out/pytest_gelu_$T.log; exit 1; }
tail -2 gpurun_out/pytest_gelu_$T.log
for L in mae_clip_amd/libmaeclip_base.so mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_base.so mae_clip_amd/libmaeclip.so; do
  echo "== $L"
  MAECLIP_LIB=$PWD/$L GEMM_SET=epi timeout -k 10 300 python -u tools/gemm_bench.py 2>/dev/null | grep "^{" | grep "gelu" || exit 1
done > gpurun_out/gemm_gelu2_ab_$T.txt
cat gpurun_out/gemm_gelu2_ab_$T.txt
timeout -k 10 900 bash tools/ab_bench.sh mae_clip_amd/libmaeclip_base.so mae_clip_amd/libmaeclip.so 2 > gpurun_out/step_gelu2_ab_$T.txt 2>&1 || { cat gpurun_out/step_gelu2_ab_$T.txt; exit 1; }
cat gpurun_out/step_gelu2_ab_$T.txt
