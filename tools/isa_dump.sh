#!/bin/bash
# Disassemble the gfx950 code object of a built wc_*.o (fat binary section),
# one kernel's body per symbol; addresses and comments stripped so two builds
# compare with diff.  usage: tools/isa_dump.sh obj.o > out.s
set -e
LL=/opt/rocm/lib/llvm/bin
t=$(mktemp -d)
$LL/llvm-objcopy --dump-section=.hip_fatbin=$t/fat "$1"
$LL/clang-offload-bundler --type=o --unbundle --input=$t/fat --output=$t/co --targets=hipv4-amdgcn-amd-amdhsa--gfx950
$LL/llvm-objdump -d --no-show-raw-insn $t/co | sed -E 's/^ *[0-9a-f]+: *//; s/ *\/\/.*$//; s/<[^>]*\+0x[0-9a-f]+>//'
rm -rf $t
