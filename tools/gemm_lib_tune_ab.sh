#!/bin/bash
# hipBLASLt algorithm per shape: the heuristic's first (default) vs the fastest
# of its first 16 candidates timed once per shape (MAECLIP_GEMM_LIB_TUNE=1);
# vendor GEMM tests with tuning, then the whole C2 step, same box.
set -o pipefail
MAECLIP_GEMM_LIB_TUNE=1 timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "vendor" --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
for r in 1 2 3; do
  for t in 0 1; do
    v=$(MAECLIP_GEMM_LIB_TUNE=$t timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --no-u8-leg --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "MAECLIP_GEMM_LIB_TUNE=$t $v"
  done
done
