#!/bin/bash
# HBM traffic of the C2 decoder's grouped weight-gradient launch (bench.py's
# dominant kernel) from rocprofv3 PMC counters: kernel trace, then FETCH_SIZE and
# WRITE_SIZE in separate passes (MI355X_MICROARCH.md §HBM; FETCH_SIZE doubled on
# gfx950). usage: TAG=name bash tools/wgrad_pmc.sh
set -o pipefail
export TMPDIR=/tmp
TAG="${TAG:-wg}"
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python tools/wgrad_one.py 10 > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$ctr -o run -- \
    python tools/wgrad_one.py 6 > $OUT/$ctr.log 2>&1 || { tail -20 $OUT/$ctr.log; exit 1; }
done
python tools/pmc_summary.py $OUT --wgrad
