#!/bin/bash
# Micro-batch count per stack width (encoder D = 768, decoder D = 512), same box,
# two rounds: MAECLIP_MB_D<width> overrides config.stack_microbatches.
set -o pipefail
for r in 1 2; do
  for cfg in "2 2" "1 1" "1 2" "2 1"; do
    set -- $cfg
    v=$(MAECLIP_MB_D768=$1 MAECLIP_MB_D512=$2 timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "enc=$1 dec=$2 $v"
  done
done
