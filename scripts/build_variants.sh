#!/bin/bash
# Diagnostic: build library variants into build/ for scripts/gpu_ab.sh.
#   build/base.so      the committed sources at REF (default HEAD)
#   build/cur.so       the working tree
#   build/<name>.so    the working tree with extra flags, VARIANTS="name:flags;..."
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REF=${REF:-HEAD}
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off"
SRCS="rb_kernels.hip rb_balls.hip rb_p2p.hip rb_capi.hip"
mkdir -p "$ROOT/build"
rm -f "$ROOT"/build/*.so
TMP=$(mktemp -d)
mkdir -p "$TMP/rigidbody-simulation_amd/csrc" "$TMP/include"
for f in $SRCS rb_device.hpp rb_grid.hpp rb_internal.hpp rb_boxes.hpp; do
  git -C "$ROOT" show "$REF:rigidbody-simulation_amd/csrc/$f" > "$TMP/rigidbody-simulation_amd/csrc/$f"
done
git -C "$ROOT" show "$REF:include/rbhip.h" > "$TMP/include/rbhip.h"
(cd "$TMP/rigidbody-simulation_amd/csrc" && /opt/rocm/bin/hipcc $FLAGS -o "$ROOT/build/base.so" $SRCS) &
cd "$ROOT/rigidbody-simulation_amd/csrc"
/opt/rocm/bin/hipcc $FLAGS -o "$ROOT/build/cur.so" $SRCS &
IFS=";" read -ra V <<< "${VARIANTS:-}"
for v in "${V[@]}"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc $FLAGS $flags -o "$ROOT/build/$name.so" $SRCS &
done
wait
rm -rf "$TMP"
ls "$ROOT/build"
