#!/bin/bash
# Round 6: non-temporal (streaming) loads of the cells in K1.  nts32 = only the S32 fast
# tile (every C2 / C5 / f32_64 unit); ntall = every K1 cell load (fast, generic, prefetch).
# Round 2 measured NT on every load at -3 % K1 (within spread) and +8 % on the 32^3 emit.
# Prediction: the cells are read once, so NT keeps the staged coefficients (read back by the
# emit) in L2 / MALL: nts32 K1 equal to -3 %, emit equal to -5 % at C2; C4 (not S32) unchanged.
for r in 1 2 3; do
  for v in base nts32 ntall; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    for w in "1024 64 f64 0.999" "512 128 f32 0.9999" "1024 64 f32 0.999" "80 c3 f64 0.999"; do
      echo "$v $w"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench $w 10 2 0 0 || exit 1
    done
  done
done
