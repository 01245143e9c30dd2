#!/bin/bash
# Round 6: K1 specialised for the 16 x 4 x 16-block shape of the 32^3 units (s16_ok; gpu_sq_groups.txt:
# the generic tile issues 1.9x the instructions per cell of the S32 body).  head = the sources before.
# Prediction: the 32^3 class's K1 -15-25 % (C4 mask 4: 0.83 -> ~0.65 ms), C4 -1 %, C3 -0.5-1 %;
# C2 / C5 / f32_64 (S32 units) unchanged.
for r in 1 2 3; do
  for v in head s16; do
    L=tools/variants/$v; [ $v = s16 ] && L=wavelet-compression_amd/lib
    echo "$v m4";  WCB_C3_MASK=4 LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
    echo "$v c4";  LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
    echo "$v c3";  LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 10 2 3 0 || exit 1
    echo "$v c2";  LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 10 2 0 0 || exit 1
    echo "$v f32"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f32 0.999 10 2 0 0 || exit 1
    echo "$v c5";  LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 512 128 f32 0.9999 10 2 0 0 || exit 1
  done
done
