#!/bin/bash
# grouped weight-gradient body: pin masks (GEMM4_PIN_GRP 0 = main build, 1, 3)
# -- launch time alone, then the whole step (same box)
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r5}
for L in mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_pg1.so mae_clip_amd/libmaeclip_pg3.so mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_pg1.so mae_clip_amd/libmaeclip_pg3.so; do
  echo "== $L $(MAECLIP_LIB=$PWD/$L timeout -k 10 200 python -u tools/wgrad_one.py 2>/dev/null | tail -1)"
done > gpurun_out/wgrad_pinmask_ab_$T.txt || exit 1
cat gpurun_out/wgrad_pinmask_ab_$T.txt
MAECLIP_LIB=$PWD/mae_clip_amd/libmaeclip_pg3.so timeout -k 10 300 python -u tools/gemm_race_screen.py > gpurun_out/race_pg3_$T.jsonl 2>&1 || { cat gpurun_out/race_pg3_$T.jsonl; exit 1; }
timeout -k 10 900 bash tools/ab_bench.sh mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_pg3.so 2 > gpurun_out/step_pinmask_ab_$T.txt 2>&1 || { cat gpurun_out/step_pinmask_ab_$T.txt; exit 1; }
cat gpurun_out/step_pinmask_ab_$T.txt
