#!/bin/bash
# Kernel resource usage (VGPRs, SGPRs, LDS, scratch) of a built object's gfx950 code object.
# Usage: scripts/kres.sh mcmc_colorer_amd/build/mcmc_sweep.hip.o [kernel-name-regex]
set -e
T=$(mktemp -d)
L=/opt/rocm/lib/llvm/bin
$L/llvm-objcopy --dump-section .hip_fatbin=$T/fat.bin "$1" /dev/null
$L/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/dev.co
$L/llvm-readelf --notes $T/dev.co > $T/notes.txt
python3 - "$T/notes.txt" "${2:-.}" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
for blk in txt.split("- .agpr_count")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk).group(1)
    if not pat.search(name): continue
    g = lambda k: (re.search(r"\." + k + r":\s+(\S+)", blk) or [None, "?"])[1]
    print(f"{name[:90]:90s} vgpr={g('vgpr_count')} sgpr={g('sgpr_count')} lds={g('group_segment_fixed_size')} scratch={g('private_segment_fixed_size')}")
PY
rm -rf $T
