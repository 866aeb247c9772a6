#!/bin/bash
# Time the v6 main loop's streams apart (diagnostic builds of gemm6.hip):
# full kernel, no MFMA (DMA + LDS reads), no LDS reads (DMA + MFMA), DMA only.
set -o pipefail
for L in libmaeclip.so libmaeclip_v6nomfma.so libmaeclip_v6noread.so libmaeclip_v6dma.so; do
  echo "== $L"
  MAECLIP_LIB=$PWD/mae_clip_amd/$L MAECLIP_GEMM_V6=1 timeout -k 10 200 python -u tools/gemm6_probe.py child || exit 1
done
