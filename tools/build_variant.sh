#!/bin/bash
# Build a variant of libmaeclip for same-box A/B runs (tools/ab_bench.sh):
#   bash tools/build_variant.sh NAME [PATCH|-] [EXTRA_HIPFLAGS...]
# copies mae_clip_amd/csrc + include into build/var_NAME, applies PATCH (if
# given), compiles every .hip with the Makefile's flags plus EXTRA_HIPFLAGS and
# links mae_clip_amd/libmaeclip_NAME.so (git-ignored; it travels with gpurun).
set -e
NAME=$1; PATCH=${2:--}; shift; shift || true
ROOT=$(cd "$(dirname "$0")/.." && pwd)
V=$ROOT/build/var_$NAME
rm -rf "$V"; mkdir -p "$V/mae_clip_amd" "$V/obj"
cp -r "$ROOT/mae_clip_amd/csrc" "$V/mae_clip_amd/"; cp -r "$ROOT/include" "$V/"
if [ "$PATCH" != "-" ]; then (cd "$V" && patch -s -p1 < "$ROOT/$PATCH"); fi
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-function $*"
pids=()
for f in "$V"/mae_clip_amd/csrc/*.hip; do
  b=$(basename "$f" .hip)
  /opt/rocm/bin/hipcc $FLAGS -c "$f" -o "$V/obj/$b.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$V"/obj/*.o -o "$ROOT/mae_clip_amd/libmaeclip_$NAME.so"
echo "built mae_clip_amd/libmaeclip_$NAME.so"
