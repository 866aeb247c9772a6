#!/bin/bash
# A/B attention kernels: baseline library (mae_clip_amd/libmaeclip_base.so) vs the
# in-tree build (tools/attn_bench.py), then the step bench on the in-tree build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in base new; do
  if [ $lib = base ]; then L=mae_clip_amd/libmaeclip_base.so; else L=mae_clip_amd/libmaeclip.so; fi
  echo "== $lib"
  MAECLIP_LIB=$PWD/$L timeout -k 10 200 python tools/attn_bench.py > gpurun_out/abattn_$lib.txt 2>&1 || { tail -20 gpurun_out/abattn_$lib.txt; exit 1; }
  grep '^{' gpurun_out/abattn_$lib.txt
done
if [ -z "$NO_BENCH" ]; then
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err || { tail -30 gpurun_out/bench_ab.err; exit 1; }
cat gpurun_out/bench_ab.json
fi
