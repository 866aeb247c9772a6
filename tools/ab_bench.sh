#!/bin/bash
# Same-box A/B of whole-step throughput across library builds, alternating:
# usage bash tools/ab_bench.sh libA.so libB.so [rounds]
set -o pipefail
mkdir -p gpurun_out
R=${3:-2}
for r in $(seq 1 $R); do
  for L in "$1" "$2"; do
    v=$(MAECLIP_LIB=$PWD/$L timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$L $v"
  done
done
