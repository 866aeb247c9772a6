#!/bin/bash
# attention tests (all bwd variants), then C4 / C2 bench with the two-image bwd off vs auto
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp8_gpu.py -q -m gpu -k "attention or fp8" --timeout 120 --timeout-method thread > gpurun_out/pt_attn.log 2>&1
rc=$?; tail -3 gpurun_out/pt_attn.log; grep -E "FAILED" gpurun_out/pt_attn.log | head
[ $rc -eq 0 ] || exit $rc
for cfg in "c4 fp8"; do
  set -- $cfg
  for two in auto; do
    if [ $two = auto ]; then unset MAECLIP_ATTN_TWO; else export MAECLIP_ATTN_TWO=$two; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-parity --config $1 --precision $2 > gpurun_out/b_$1_$two.json 2> gpurun_out/b_$1_$two.err || { tail -20 gpurun_out/b_$1_$two.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/b_$1_$two.json'));print('$1 two=$two', d['value'], d['ms_per_step'])"
  done
done
unset MAECLIP_ATTN_TWO
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4two -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-parity --no-kernel-timer --config c4 --precision fp8 > gpurun_out/prof_c4two.log 2>&1 || { tail -30 gpurun_out/prof_c4two.log; exit 1; }
f=$(find gpurun_out/prof_c4two -name "*kernel_stats.csv" | head -1)
python tools/prof_summary.py "$f" 8 14 | grep -E "attn|total|quant|wq_|gemm4_f8"
