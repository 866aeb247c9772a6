#!/bin/bash
# C4 (ViT-L/14@336, B=128) fp8: fp8 no-epilogue / residual GEMMs on the vendor library
# (MAECLIP_GEMM_LIB_FP8=1, default) vs the own fp8 kernel (=0); bf16 line for the ratio.
set -o pipefail
for r in 1 2; do
  for p in 0 1; do
    v=$(MAECLIP_GEMM_LIB_FP8=$p timeout -k 10 300 python -u bench.py --config c4 --precision fp8 --no-cpu-baseline --no-parity --no-u8-leg --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "c4 fp8 MAECLIP_GEMM_LIB_FP8=$p $v"
  done
  v=$(timeout -k 10 300 python -u bench.py --config c4 --precision bf16 --no-cpu-baseline --no-parity --no-u8-leg --steps 10 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
  echo "c4 bf16 $v"
done
