#!/bin/bash
# Disassembly of one kernel of a built object's gfx950 code object.
# Usage: scripts/kisa.sh mcmc_colorer_amd/build/mcmc_sweep.hip.o <mangled-kernel-name> > out.s
set -e
T=$(mktemp -d)
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section .hip_fatbin=$T/fat.bin "$1" /dev/null
$L/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/dev.co
$L/llvm-objdump -d --no-show-raw-insn --disassemble-symbols="$2" $T/dev.co
rm -rf $T
