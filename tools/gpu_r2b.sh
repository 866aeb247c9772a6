#!/bin/bash
# tests + bench (graph) + bench --dp (eager DP path at N=1) + PMC breakdown of the dominant GEMM
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2b} NO_BENCH=1 PYT_LIMIT=600 bash tools/gpu_r2.sh; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_${TAG:-r2b}.json 2> gpurun_out/bench_${TAG:-r2b}.err || { tail -30 gpurun_out/bench_${TAG:-r2b}.err; exit 1; }
cat gpurun_out/bench_${TAG:-r2b}.json
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --dp > gpurun_out/bench_${TAG:-r2b}_dp.json 2> gpurun_out/bench_${TAG:-r2b}_dp.err || { tail -30 gpurun_out/bench_${TAG:-r2b}_dp.err; exit 1; }
cat gpurun_out/bench_${TAG:-r2b}_dp.json
bash tools/pmc_gemm.sh 50432 2048 512 0 1 5 > gpurun_out/pmc_${TAG:-r2b}.txt 2>&1
cat gpurun_out/pmc_${TAG:-r2b}.txt
exit $rc
