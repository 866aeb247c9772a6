#!/bin/bash
# Same-box scan of the micro-batch count (config.stack_microbatches) and the
# HIP hardware-queue count, alternating, whole-step img/s (bench.py quick line).
set -o pipefail
for r in 1 2; do
  for cfg in "1 4" "2 4" "4 4" "2 8" "4 8"; do
    set -- $cfg
    v=$(GPU_MAX_HW_QUEUES=$2 timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --no-u8-leg --steps 20 --microbatches $1 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "microbatches=$1 hw_queues=$2 $v"
  done
done
