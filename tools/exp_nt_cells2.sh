#!/bin/bash
# Round 6, second call: base vs ntall (nontemporal cell loads in every K1 form) vs ntep (ntall with
# the emit's staged-coefficient loads plain again), forward only, plus the global-threshold mode at C4.
# Question: the first call (exp_nt_cells.sh) showed K1 -10 % and the emit +7 % at C2 with NT cell
# loads; does the emit's own NT load cause its loss?  Prediction: ntep emit back to base's 0.205 ms
# with K1 still -10 %: C2 forward -8 %.
for r in 1 2 3 4; do
  for v in base ntall ntep; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    for w in "1024 64 f64 0.999" "512 128 f32 0.9999" "1024 64 f32 0.999" "80 c3 f64 0.999"; do
      echo "$v $w"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench $w 10 2 0 0 || exit 1
    done
    echo "$v c4hist"; WCB_HIST=0.7 LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
  done
done
