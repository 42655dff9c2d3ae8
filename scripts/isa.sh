#!/bin/bash
# Diagnostic: disassemble one kernel of rb_kernels.hip (gfx950) to /tmp/<name>.s
# usage: scripts/isa.sh MANGLED_NAME OUT [extra hipcc flags]
set -eu
cd "$(dirname "$0")/../rigidbody-simulation_amd/csrc"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off ${3:-} --cuda-device-only -c -o /tmp/kdev.o rb_kernels.hip
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=/tmp/kdev.o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=/tmp/kdev_gfx950.o
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn --disassemble-symbols="$1" /tmp/kdev_gfx950.o > "$2"
wc -l "$2"
