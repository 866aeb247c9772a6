#!/bin/bash
# Same-box whole-step A/B across environment settings, alternating rounds:
#   ROUNDS=2 bash tools/env_ab.sh "MAECLIP_GEMM_SK=0" "MAECLIP_GEMM_SK=0 MAECLIP_MB_D768=1" ...
# ("-" = no extra variable). One line per run: setting, img/s, ms/step.
set -o pipefail
R=${ROUNDS:-2}
for r in $(seq 1 $R); do
  for cfg in "$@"; do
    envs=(); [ "$cfg" != "-" ] && read -r -a envs <<< "$cfg"
    v=$(env "${envs[@]}" timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "[$cfg] $v"
  done
done
