#!/bin/bash
# Attention forward variants: the default build vs mae_clip_amd/libmaeclip_${VAR}.so
# (VAR=nodma: -DATTN_DMA=0, the register path for the K / V images; VAR=noqimg:
# -DATTN_QIMG=0, Q fragments from global per tile): attention tests, kernel times
# at the production shapes, whole-step A/B, PMC of the C2 decoder forward.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q -k "attn or attention" --timeout 120 \
  --timeout-method thread > gpurun_out/attn_dma_tests.txt 2>&1 || { tail -30 gpurun_out/attn_dma_tests.txt; exit 1; }
tail -2 gpurun_out/attn_dma_tests.txt
for L in libmaeclip.so libmaeclip_${VAR:-nodma}.so; do
  echo "== $L"
  MAECLIP_LIB=$PWD/mae_clip_amd/$L timeout -k 10 180 python -u tools/attn_bench.py 2>&1 | grep -v "^$" | tail -14 || exit 1
done
timeout -k 10 900 bash tools/ab_bench.sh mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_${VAR:-nodma}.so 2 || exit 1
PMCDIR=gpurun_out/pmca_${VAR:-dma} timeout -k 10 400 bash tools/pmc_attn.sh 256 197 16 32 0 > gpurun_out/pmc_attn_dec_fwd_${VAR:-dma}.txt 2>&1 || exit 1
cat gpurun_out/pmc_attn_dec_fwd_${VAR:-dma}.txt
