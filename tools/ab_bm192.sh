#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -k "gemm" > gpurun_out/pt_bm.log 2>&1; rc=$?
tail -3 gpurun_out/pt_bm.log
[ $rc -eq 0 ] || { grep -E "^E|assert" gpurun_out/pt_bm.log | head -20; exit 1; }
for bm in 256 0; do echo "== BM=$bm"; MAECLIP_GEMM_BM=$bm GEMM_SET=epi timeout -k 10 200 python tools/gemm_bench.py 2>/dev/null | grep '^{' | grep enc | cut -c1-150; done
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pt_model.log 2>&1; tail -2 gpurun_out/pt_model.log
for bm in 256 0 256 0; do MAECLIP_GEMM_BM=$bm timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('BM=$bm', d['value'], d['ms_per_step'])"; done
