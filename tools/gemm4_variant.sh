#!/bin/bash
# Diagnostic variant of libmaeclip that differs only in gemm4.hip's flags:
#   bash tools/gemm4_variant.sh NAME [EXTRA_HIPFLAGS...]
# compiles gemm4.hip with the Makefile's flags + EXTRA_HIPFLAGS, links it with
# the other objects of the current build (make first) into
# mae_clip_amd/libmaeclip_NAME.so (git-ignored; it travels with gpurun).
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
O=$ROOT/build/g4var_$NAME
mkdir -p "$O"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-function "$@" \
  -c "$ROOT/mae_clip_amd/csrc/gemm4.hip" -o "$O/gemm4.o"
objs=$(ls "$ROOT"/build/obj/*.o | grep -v '/gemm4.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "$O/gemm4.o" -o "$ROOT/mae_clip_amd/libmaeclip_$NAME.so"
echo "built mae_clip_amd/libmaeclip_$NAME.so"
