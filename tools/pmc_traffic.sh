#!/bin/bash
# HBM traffic of one GEMM shape from rocprofv3 PMC counters, one counter group
# per pass (MI355X_MICROARCH.md §HBM: FETCH_SIZE costs 3 TCC slots, WRITE_SIZE 2,
# so they cannot share a pass; FETCH_SIZE reads 1/2 of a wide streaming read on
# gfx950 and is doubled; WRITE_SIZE is exact for 16-B stores).
# usage: TAG=name bash tools/pmc_traffic.sh M N K la lb epi
set -o pipefail
export TMPDIR=/tmp
TAG="${TAG:-pmc}"
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python tools/gemm_one.py "$@" 20 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$ctr -o run -- \
    python tools/gemm_one.py "$@" 20 > $OUT/$ctr.log 2>&1 || { tail -20 $OUT/$ctr.log; exit 1; }
done
python tools/pmc_summary.py $OUT "$@"
