#!/bin/bash
# tokens_bwd_pos / MAE HBM kernels across library builds on ONE box:
# usage bash tools/ab_tokens.sh tag1:lib1.so tag2:lib2.so ... (kernel stats in gpurun_out/tok_<tag>)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "tokens or mae or unshuffle" > gpurun_out/tok_t.txt 2>&1 && tail -1 gpurun_out/tok_t.txt || exit 1
for TL in "$@"; do
  T=${TL%%:*}; L=${TL#*:}
  MAECLIP_LIB=$PWD/$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tok_$T -o run -- python -u bench.py --no-cpu-baseline --no-parity --steps 10 --warmup 3 > gpurun_out/tok_bench_$T.json 2> gpurun_out/tok_bench_$T.err || exit 1
  echo "$T $(python -c "import json;d=json.load(open('gpurun_out/tok_bench_$T.json'));print(d['value'], d['ms_per_step'])")"
done
