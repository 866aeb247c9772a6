#!/bin/bash
# C4 fp8 (decoder in fp8): decoder micro-batch chains 2 (default) vs 1, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for d in 2 1; do
    v=$(MAECLIP_MB_D512=$d timeout -k 10 300 python -u bench.py --config c4 --precision fp8 --no-cpu-baseline \
        --no-parity --no-u8-leg --steps 10 2>gpurun_out/c4decmb.err \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") \
      || { tail -20 gpurun_out/c4decmb.err; exit 1; }
    echo "dec_mb=$d $v"
  done
done
