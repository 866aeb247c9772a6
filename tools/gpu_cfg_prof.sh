#!/bin/bash
# bench of each config in $CFGS (no cpu baseline / parity), then a kernel-trace
# profile of $PROF (a config name) when set
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CFGS:-c2}; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline --no-parity > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || { tail -20 gpurun_out/bench_$c.err; exit 1; }
  python -c "import json; r=json.load(open('gpurun_out/bench_$c.json')); print('$c', r['value'], r['ms_per_step'], r['roofline']['achieved'], r['roofline'].get('kernel'))"
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$PROF -o run --output-format csv -- python bench.py --config $PROF --steps 3 --warmup 2 --no-cpu-baseline --no-parity --no-kernel-timer > gpurun_out/prof_$PROF.log 2>&1 || exit $?
  find gpurun_out/prof_$PROF -name "*stats*" | head
fi
