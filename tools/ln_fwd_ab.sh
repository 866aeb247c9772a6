#!/bin/bash
# LayerNorm forward variants: isolated (tools/ln_probe.py) per library, the LN
# tests per variant, then the whole C2 step (tools/ab_bench.sh style), same box.
# The variants were built with tools/build_variant.sh NAME - -DLN_FWD_PERSIST=1
# -DLN_FWD_WGS=2048|1024 from a layernorm.hip that has since dropped that macro
# (measured slower: profiles/r04/ln_fwd_persistent_ab_r4ak.txt).
set -o pipefail
mkdir -p gpurun_out
for L in libmaeclip.so libmaeclip_lnp2k.so libmaeclip_lnp1k.so; do
  echo "== $L"
  MAECLIP_LIB=$PWD/mae_clip_amd/$L timeout -k 10 200 python -u tools/ln_probe.py 2>/dev/null | grep '^{' || exit 1
done
for L in libmaeclip_lnp2k.so libmaeclip_lnp1k.so; do
  MAECLIP_LIB=$PWD/mae_clip_amd/$L timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "layernorm or ln_" --timeout 120 --timeout-method thread 2>&1 | tail -1 || exit 1
done
for r in 1 2; do
  for L in libmaeclip.so libmaeclip_lnp2k.so libmaeclip_lnp1k.so; do
    v=$(MAECLIP_LIB=$PWD/mae_clip_amd/$L timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-parity --no-u8-leg --steps 20 2>/dev/null \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") || exit 1
    echo "$L $v"
  done
done
