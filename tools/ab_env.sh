#!/bin/bash
# A/B env settings on the epilogue GEMM shapes and the step: AB="VAR=a VAR=b ..."
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for kv in $AB; do
  echo "== $kv"
  env $kv GEMM_SET=${GEMM_SET:-epi} timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/abe.txt 2>&1 || { tail -20 gpurun_out/abe.txt; exit 1; }
  python -c "
import json
for l in open('gpurun_out/abe.txt'):
    if l.startswith('{'):
        r=json.loads(l); print(f\"{r['ours_us']:8.1f}us {r['ours_tflops']:7.1f}TF  {r['name']}\")"
  if [ -n "$STEP" ]; then
    env $kv timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > gpurun_out/abe.json 2> gpurun_out/abe.err || { tail -20 gpurun_out/abe.err; exit 1; }
    python -c "import json; r=json.load(open('gpurun_out/abe.json')); print('STEP', r['value'], r['ms_per_step'])"
  fi
done
