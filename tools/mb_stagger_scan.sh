#!/bin/bash
# Same-box scan of the micro-batch stagger (MAECLIP_MB_STAGGER=k: micro-batch 1
# starts a block after micro-batch 0 has issued k of its launches), whole C2 step.
set -o pipefail
for r in 1 2; do
  for k in 0 2 3 4 5; do
    v=$(MAECLIP_MB_STAGGER=$k timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "MAECLIP_MB_STAGGER=$k $v"
  done
done
