#!/bin/bash
# one gpurun call: bench (with cpu baseline + parity) then a rocprofv3 kernel-trace of a short bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
cat gpurun_out/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-parity --no-kernel-timer > gpurun_out/prof.log 2>&1 || exit $?
find gpurun_out/prof -name "*stats*" | head
