#!/bin/bash
# Per-shape GEMM table of one eager C2 step (HIP events per launch) + the
# SQ/TCC PMC breakdown of the dominant GEMM shape (separate passes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG="${TAG:-gt}"
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --gemm-table --steps 3 --warmup 2 ${BENCH_ARGS} \
  > gpurun_out/gemm_table_${TAG}.json 2> gpurun_out/gemm_table_${TAG}.txt || { tail -30 gpurun_out/gemm_table_${TAG}.txt; exit 1; }
grep -A60 "GEMM total" gpurun_out/gemm_table_${TAG}.txt
if [ -n "$PMC" ]; then
  bash tools/pmc_gemm.sh $PMC > gpurun_out/pmc_${TAG}.txt 2>&1; rc=$?
  cat gpurun_out/pmc_${TAG}.txt
  exit $rc
fi
