#!/bin/bash
# Pinned MFMA clusters (gemm4.hip pin_quad) vs the compiler's split clusters
# (GEMM4_NO_PIN) vs pinned except the grouped weight gradients: race screen,
# per-shape GEMM times, grouped weight-gradient launch time, whole step.
set -o pipefail
mkdir -p gpurun_out
T=${TAG:-r5}
timeout -k 10 300 python -u tools/gemm_race_screen.py > gpurun_out/race_pin_$T.jsonl 2>&1 || { cat gpurun_out/race_pin_$T.jsonl; exit 1; }
tail -3 gpurun_out/race_pin_$T.jsonl
for L in mae_clip_amd/libmaeclip_nopin.so mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_nopin.so mae_clip_amd/libmaeclip.so; do
  echo "== $L"
  MAECLIP_LIB=$PWD/$L GEMM_SET=epi timeout -k 10 300 python -u tools/gemm_bench.py 2>/dev/null | grep "^{" || exit 1
  MAECLIP_LIB=$PWD/$L GEMM_SET=sq timeout -k 10 300 python -u tools/gemm_bench.py 2>/dev/null | grep "^{" || exit 1
done > gpurun_out/gemm_pin_ab_$T.txt
for L in mae_clip_amd/libmaeclip_nopin.so mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_pinnogrp.so mae_clip_amd/libmaeclip_nopin.so mae_clip_amd/libmaeclip.so mae_clip_amd/libmaeclip_pinnogrp.so; do
  echo "== $L $(MAECLIP_LIB=$PWD/$L timeout -k 10 200 python -u tools/wgrad_one.py 2>/dev/null | tail -1)"
done > gpurun_out/wgrad_pin_ab_$T.txt
cat gpurun_out/wgrad_pin_ab_$T.txt
timeout -k 10 900 bash tools/ab_bench.sh mae_clip_amd/libmaeclip_nopin.so mae_clip_amd/libmaeclip.so 2 > gpurun_out/step_pin_ab_$T.txt 2>&1 || { cat gpurun_out/step_pin_ab_$T.txt; exit 1; }
timeout -k 10 500 bash tools/ab_bench.sh mae_clip_amd/libmaeclip_pinnogrp.so mae_clip_amd/libmaeclip.so 1 >> gpurun_out/step_pin_ab_$T.txt 2>&1 || { cat gpurun_out/step_pin_ab_$T.txt; exit 1; }
cat gpurun_out/step_pin_ab_$T.txt
