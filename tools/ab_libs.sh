#!/bin/bash
# A/B the GEMM epilogue shapes across library builds on ONE box: usage bash tools/ab_libs.sh lib1.so lib2.so ...
set -o pipefail
mkdir -p gpurun_out
for L in "$@"; do
  echo "== $L"
  MAECLIP_LIB=$PWD/$L GEMM_SET=epi timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null | grep '^{' | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(f\"{d['name']:16s} epi{d['epi']} {d['ours_us']:8.1f} us {d['ours_tflops']:7.1f} TF/s\")"
done
