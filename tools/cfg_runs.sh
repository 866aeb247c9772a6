#!/bin/bash
# C1 / C4 (bf16, fp8) bench lines + a kernel profile of C4 fp8 (one call)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r3}
for c in "c1 bf16" "c4 bf16" "c4 fp8"; do
  set -- $c
  timeout -k 10 400 python -u bench.py --config $1 --precision $2 --no-cpu-baseline --no-parity --no-u8-leg --steps 10 \
    > gpurun_out/${1}_${2}_${T}.json 2> gpurun_out/${1}_${2}_${T}.err || { tail -20 gpurun_out/${1}_${2}_${T}.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/${1}_${2}_${T}.json').read().strip().splitlines()[-1]); print('$1 $2', d['value'], d['ms_per_step'])"
done
if [ -n "$PROF4" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4fp8_${T} -o run --output-format csv -- \
    python bench.py --config c4 --precision fp8 --no-cpu-baseline --no-parity --no-u8-leg --steps 5 > gpurun_out/prof_c4fp8_${T}.log 2>&1 || exit 1
fi
