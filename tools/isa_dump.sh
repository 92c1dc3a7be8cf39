#!/bin/bash
# Disassemble the gfx950 code object embedded in a hipcc object file: tools/isa_dump.sh x.o out.s
# (used to show a source cleanup leaves the product kernels' machine code unchanged)
set -e
LLVM=/opt/rocm/lib/llvm/bin
tmp=$(mktemp -d)
$LLVM/llvm-objcopy -O binary --only-section=.hip_fatbin "$1" $tmp/fat.bin
$LLVM/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$tmp/fat.bin --output=$tmp/dev.co
$LLVM/llvm-objdump -d --no-show-raw-insn $tmp/dev.co | sed -e 's/^ *[0-9a-f]*://' > "$2"
rm -rf $tmp
