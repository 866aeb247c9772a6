#!/bin/bash
# A/B the GEMM epilogue shapes: baseline library (mae_clip_amd/libmaeclip_base.so) vs the
# in-tree build, then the GEMM parity tests and the step bench on the in-tree build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in base new; do
  echo "== $lib"
  if [ $lib = base ]; then L=mae_clip_amd/libmaeclip_base.so; else L=mae_clip_amd/libmaeclip.so; fi
  MAECLIP_LIB=$PWD/$L GEMM_SET=${GEMM_SET:-epi} timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/ab_$lib.txt 2>&1 || { tail -20 gpurun_out/ab_$lib.txt; exit 1; }
  cat gpurun_out/ab_$lib.txt | grep '^{'
done
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -30 gpurun_out/bench_ab.err; exit 1; }
cat gpurun_out/bench_ab.json
