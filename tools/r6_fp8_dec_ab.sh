#!/bin/bash
# fp8 decoder A/B (MAECLIP_FP8_DECODER=1 vs 0): C4 fp8 parity test with the
# decoder on fp8 GEMMs (parity record to gpurun_out/), then alternating C4 fp8
# bench lines.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MAECLIP_PARITY_OUT=$PWD/gpurun_out/parity_fp8dec.jsonl MAECLIP_FP8_DECODER=1 timeout -k 10 300 \
  python -u -m pytest tests/test_fp8_gpu.py -m gpu -x -q -k "vitl14" --timeout 240 --timeout-method thread \
  > gpurun_out/fp8dec_tests.txt 2>&1 || { tail -30 gpurun_out/fp8dec_tests.txt; cat gpurun_out/parity_fp8dec.jsonl; exit 1; }
tail -2 gpurun_out/fp8dec_tests.txt
cat gpurun_out/parity_fp8dec.jsonl
for r in 1 2; do
  for d in 1 0; do
    v=$(MAECLIP_FP8_DECODER=$d timeout -k 10 300 python -u bench.py --config c4 --precision fp8 --no-cpu-baseline \
        --no-parity --no-u8-leg --steps 10 2>gpurun_out/fp8dec_bench.err \
        | python -c "import sys, json; d = json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])") \
      || { tail -20 gpurun_out/fp8dec_bench.err; exit 1; }
    echo "fp8_decoder=$d $v"
  done
done
