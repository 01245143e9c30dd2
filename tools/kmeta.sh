#!/bin/bash
# Register metadata of the kernels of one source: tools/kmeta.sh <stem> [name filter] [-DMACRO=v ...]
# (vgpr_count, vgpr_spill_count, private segment, sgpr_count) — the spill test's source, readable.
# Without -D options: the built object; with them: that source compiled with them (product flags).
set -e
L=/opt/rocm/lib/llvm/bin
CS=wavelet-compression_amd/csrc
stem=$1; filt="${2:-.}"; shift; shift || true
t=$(mktemp -d)
o=wavelet-compression_amd/build/$stem.o
if [ $# -gt 0 ]; then
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-gpu-flush-denormals-to-zero \
    -fno-fast-math -Iinclude -I$CS "$@" -c $CS/$stem.hip -o $t/o.o
  o=$t/o.o
fi
$L/llvm-objcopy --dump-section=.hip_fatbin=$t/f $o
$L/clang-offload-bundler --type=o --unbundle --input=$t/f --output=$t/co --targets=hipv4-amdgcn-amd-amdhsa--gfx950
$L/llvm-readelf --notes $t/co | grep -E "^\s+\.(name|vgpr_count|vgpr_spill_count|private_segment_fixed_size|sgpr_count):" | \
  paste - - - - - | grep -E "$filt" | awk '{print $2, "priv", $4, "vgpr", $8, "spill", $10}' | c++filt | sed -E "s/\(.*\)/()/"
rm -rf $t
