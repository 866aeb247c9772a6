#!/bin/bash
# Quick register / spill check of gemm4.hip (one epilogue per layout:
# GEMM4_DEV_SUBSET) -> /tmp/isa/g4sub.remarks + the device .s
mkdir -p /tmp/isa/sub && cd /tmp/isa/sub || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -DGEMM4_DEV_SUBSET $EXTRA \
  -Rpass-analysis=kernel-resource-usage -save-temps -c /root/repo/mae_clip_amd/csrc/gemm4.hip -o g4sub.o > /tmp/isa/g4sub.remarks 2>&1
python3 /root/repo/tools/kernel_regs.py /tmp/isa/g4sub.remarks "${1:-gemm4_kernel|wgrad4_kernel|f8_kernel}"
