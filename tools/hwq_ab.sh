#!/bin/bash
# HIP hardware queues per process (GPU_MAX_HW_QUEUES, 4 on the box) on the whole
# C2 step: the two micro-batch chains, the side stream and the upload stream map
# onto them. Same box, alternating.
set -o pipefail
for r in 1 2 3; do
  for q in 4 8; do
    v=$(GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --no-u8-leg --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "GPU_MAX_HW_QUEUES=$q $v"
  done
done
