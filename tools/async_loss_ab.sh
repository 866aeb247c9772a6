#!/bin/bash
# Same-box A/B (3 rounds): per-step loss read before vs after queueing the next step.
set -o pipefail
for r in 1 2 3; do
  for f in "--sync-loss" ""; do
    v=$(timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-parity --steps 20 $f 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "mode=${f:-read-after-next-queued} $v"
  done
done
