#!/bin/bash
# Builds libwavelet_amd.so variants (one -D each, tuning macros only: no build
# of the product sources writes invalid results) under tools/variants/<name>/ for
# A/B runs of tools/bin/wc_bench with LD_LIBRARY_PATH (its RUNPATH yields to it).
set -e
# VSRC=<dir>: compile the kernel and C-ABI sources from a patched copy of csrc
# (diagnostic variants whose results are not valid never enter the product tree)
CS=${VSRC:-wavelet-compression_amd/csrc}
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-gpu-flush-denormals-to-zero -fno-fast-math -Iinclude -I$CS"
for spec in "$@"; do
  name="${spec%%:*}"; defs="${spec#*:}"
  out=tools/variants/$name; mkdir -p $out/obj
  for f in wc_transform wc_hist wc_compact wc_inverse wc_emit; do
    /opt/rocm/bin/hipcc $FLAGS $defs -c $CS/$f.hip -o $out/obj/$f.o &
  done
  for f in wc_common wc_plan wc_capi wc_hostpipe; do
    /opt/rocm/bin/hipcc $FLAGS $defs -c $CS/$f.cpp -o $out/obj/$f.o &
  done
  g++ -O2 -std=c++17 -fPIC -c $CS/wc_hostmem.cpp -o $out/obj/wc_hostmem.o &
  wait
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libwavelet_amd.so $out/obj/*.o -lpthread
  rm -rf $out/obj
done
