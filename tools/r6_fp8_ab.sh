#!/bin/bash
# C4 fp8 step A/B of the attention's fused fp8 copies (config.fp8_attn_q8 via
# MAECLIP_FP8_ATTN_Q8), interleaved, ROUNDS rounds; then C4 bf16 once
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r6}
for r in $(seq ${ROUNDS:-2}); do
  for m in ${MODES:-10 00 11}; do
    MAECLIP_FP8_ATTN_Q8=$m timeout -k 10 400 python -u bench.py --config c4 --precision fp8 --no-cpu-baseline --no-parity \
      --no-u8-leg --steps 10 > gpurun_out/c4ab_${m}_${r}_${TAG}.json 2> gpurun_out/c4ab_${m}_${r}_${TAG}.err \
      || { tail -20 gpurun_out/c4ab_${m}_${r}_${TAG}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/c4ab_${m}_${r}_${TAG}.json').read().strip().splitlines()[-1]); print('fp8 attn_q8=$m round $r', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 400 python -u bench.py --config c4 --precision bf16 --no-cpu-baseline --no-parity --no-u8-leg --steps 10 \
  > gpurun_out/c4ab_bf16_${TAG}.json 2> gpurun_out/c4ab_bf16_${TAG}.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/c4ab_bf16_${TAG}.json').read().strip().splitlines()[-1]); print('bf16', d['value'], d['ms_per_step'])"
