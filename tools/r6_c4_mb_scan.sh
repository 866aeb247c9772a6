#!/bin/bash
# C4 micro-batch count scan of the encoder stack (MAECLIP_MB_D1024 = chains),
# fp8 and bf16, interleaved; then C1 bf16 once
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r6}
for r in 1 2; do
  for p in fp8 bf16; do
    for s in 1 2 4; do
      MAECLIP_MB_D1024=$s timeout -k 10 400 python -u bench.py --config c4 --precision $p --no-cpu-baseline --no-parity \
        --no-u8-leg --steps 10 > gpurun_out/c4mb_${p}_${s}_${r}_${TAG}.json 2> gpurun_out/c4mb_${p}_${s}_${r}_${TAG}.err \
        || { tail -20 gpurun_out/c4mb_${p}_${s}_${r}_${TAG}.err; exit 1; }
      python -c "import json; d=json.loads(open('gpurun_out/c4mb_${p}_${s}_${r}_${TAG}.json').read().strip().splitlines()[-1]); print('c4 $p encoder chains $s round $r', d['value'], d['ms_per_step'])"
    done
  done
done
timeout -k 10 400 python -u bench.py --config c1 --no-cpu-baseline --no-parity --no-u8-leg --steps 10 \
  > gpurun_out/c1_${TAG}.json 2> gpurun_out/c1_${TAG}.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/c1_${TAG}.json').read().strip().splitlines()[-1]); print('c1 bf16', d['value'], d['ms_per_step'])"
