#!/bin/bash
# Round 6 A/B in one call (profiles/r06/experiments/gpu_split_wide.txt):
#   base    = working tree (K1 fast tiles in two LDS classes; fused-RMSE K6r on the wide-x list)
#   nosplit = one LDS class (kLdsFastA huge: the round-5 single fast launch)
#   nowide  = the fused-RMSE K6r on the 16 x 2 list (round 5)
for r in 1 2 3; do
  for v in base nosplit nowide; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    echo "$v c4ref"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
    echo "$v c4hist"; WCB_HIST=0.7 LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
    echo "$v c3rt"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 20 3 3 0 || exit 1
    echo "$v c2inv"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 0 || exit 1
  done
done
