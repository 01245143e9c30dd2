#!/bin/bash
# Round 6: nontemporal payload stores in the emit, re-tried on the round-6 K1 (nontemporal cell
# loads).  Round 5 measured them at emit +7 % (r05/experiments/gpu_nt.txt); bw_probe's 1:2 mix
# reaches 5.5 TB/s with nontemporal stores vs 5.35 plain (gpu_bw_mix.txt).
# Prediction: emit -0-3 %, the inverse after it (which reads the payloads) +0-3 %.
for r in 1 2 3; do
  for v in base ntpay; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    for w in "1024 64 f64 0.999 10 2 1" "512 128 f32 0.9999 10 2 1" "1024 64 f32 0.999 10 2 1" "80 c3 f64 0.999 10 2 0"; do
      echo "$v $w"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench $w 0 || exit 1
    done
  done
done
