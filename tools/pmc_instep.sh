#!/bin/bash
# In-step HBM traffic of the bench's dominant GEMM launch: the C2 step itself
# (eager steps, same shapes, data and stream layout as the timed run) under
# rocprofv3 -- one kernel-trace pass for durations, then FETCH_SIZE and
# WRITE_SIZE each in a pass of its own (MI355X_MICROARCH.md §HBM: they cannot
# share a pass; FETCH_SIZE is doubled on gfx950). The dominant launch is picked
# by kernel name (unique in the C2 step) and, for instantiations shared by
# several shapes, by grid size.
# usage: TAG=name [PICK=I/K] bash tools/pmc_instep.sh 'KERNEL_NAME_SUBSTRING' GRID_X "SHAPE KEY" [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG="${TAG:-instep}"
OUT=gpurun_out/pmcstep_$TAG
KN=$1; GX=$2; KEY=$3; shift 3
mkdir -p $OUT
B="bench.py --no-graph --steps 2 --warmup 1 --no-cpu-baseline --no-parity --no-u8-leg --no-kernel-timer $*"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python $B > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$ctr -o run -- python $B > $OUT/$ctr.log 2>&1 || { tail -20 $OUT/$ctr.log; exit 1; }
done
python tools/pmc_instep_summary.py $OUT "$KN" "$GX" "$KEY" "$PICK"
