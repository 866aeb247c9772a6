#!/bin/bash
# The data-parallel code path at world 1 (RCCL group, embedding all-gather,
# bucketed gradient all-reduce, captured) vs the plain step, same box, alternating.
set -o pipefail
for r in 1 2; do
  for m in "" "--dp"; do
    v=$(timeout -k 10 240 python -u bench.py $m --no-cpu-baseline --no-parity --no-u8-leg --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['rccl'])") || exit 1
    echo "bench.py ${m:-(no --dp)} $v"
  done
done
