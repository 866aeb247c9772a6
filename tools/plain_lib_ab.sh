#!/bin/bash
# Same-box A/B (3 rounds): plain bf16 GEMMs on the vendor library (MAECLIP_GEMM_LIB=1,
# the default, gemm_lib.hip) vs this library's v4 kernel (=0).
set -o pipefail
for r in 1 2 3; do
  for p in 1 3; do
    v=$(MAECLIP_GEMM_LIB=$p timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "MAECLIP_GEMM_LIB=$p $v"
  done
done
