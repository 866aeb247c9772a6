#!/bin/bash
# Whole C2 step with the GEMM epilogue's non-temporal streams varied
# (GEMM4_EPI_NT: 3 = loads + stores (default), 2 = stores only, 0 = none), same box.
set -o pipefail
for r in 1 2; do
  for L in libmaeclip.so libmaeclip_nt2.so libmaeclip_nt0.so; do
    v=$(MAECLIP_LIB=$PWD/mae_clip_amd/$L timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --no-u8-leg --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$L $v"
  done
done
