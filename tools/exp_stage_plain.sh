#!/bin/bash
# Round 6: K1 staging stores plain again (with round 6's nontemporal cell loads).
# Round 5 made them nontemporal when the cell loads were plain (K1 -2 % C2, -4 % C5).
# Prediction: with the cells now streamed, plain staged lines stay in the Infinity Cache for the
# emit: emit -3-5 %, K1 +0-2 %.
for r in 1 2 3; do
  for v in base stplain; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    for w in "1024 64 f64 0.999 10 2 1" "512 128 f32 0.9999 10 2 1" "1024 64 f32 0.999 10 2 1" "80 c3 f64 0.999 10 2 0"; do
      echo "$v $w"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench $w 0 || exit 1
    done
  done
done
