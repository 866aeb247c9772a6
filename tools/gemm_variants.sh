#!/bin/bash
# GEMM v2 tile variants vs v1 (99) on the production shapes
for v in ${VARIANTS:-1 4 99}; do
  echo "== variant $v"
  MAECLIP_GEMM_VARIANT=$v timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(f\"{r['name']:16s} {r['ours_tflops']:7.1f} TF {r['ours_us']:8.1f} us (hipBLASLt {r['hipblaslt_tflops']:7.1f})\")
" || exit 1
done
