#!/bin/bash
# VGPR / SGPR / LDS / scratch of every kernel in a hipcc object file's gfx950 code object:
# tools/kernel_resources.sh x.o [name-filter]
set -e
LLVM=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
$LLVM/llvm-objcopy -O binary --only-section=.hip_fatbin "$1" $tmp/fat.bin
$LLVM/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$tmp/fat.bin --output=$tmp/dev.co
$LLVM/llvm-readelf --notes $tmp/dev.co | python3 -c "
import sys, re
txt = sys.stdin.read()
flt = sys.argv[1] if len(sys.argv) > 1 else ''
for blk in re.split(r'\n\s*- \.agpr_count', txt)[1:]:
    name = re.search(r'\.name:\s+(\S+)', blk)
    if not name or flt not in name.group(1): continue
    g = lambda k: (re.search(r'\.' + k + r':\s+(\S+)', blk) or [None, '?'])[1]
    print(f\"{name.group(1)[:90]:90s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size'):>4} spill_v {g('vgpr_spill_count')}\")
" "${2:-}"
rm -rf $tmp
