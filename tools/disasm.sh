#!/bin/bash
# gfx950 disassembly of one built object: tools/disasm.sh OBJ OUT.s
set -e
t=$(mktemp -d)
objcopy --dump-section .hip_fatbin=$t/fb.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$t/fb.bin --output=$t/co.elf
/opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn $t/co.elf > "$2"
rm -rf $t
