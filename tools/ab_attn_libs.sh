#!/bin/bash
# attention kernel times across library builds on ONE box:
# usage bash tools/ab_attn_libs.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for L in "$@"; do
  echo "== $L"
  MAECLIP_LIB=$PWD/$L timeout -k 10 200 python tools/attn_bench.py 2>/dev/null | grep '^{' || exit 1
done
