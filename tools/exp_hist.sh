#!/bin/bash
# Round 6: where the fused-histogram K1's time goes at C4 (profiles/r06/experiments/gpu_hist_split.txt).
# base: k_transform_hist (persistent, 16 KiB LDS bins, 3 workgroups/CU) + emit at quantile 0.7;
# histA: the same kernel without the bin adds (occupancy + persistence alone);
# histC: plain LDS atomics instead of the wave-aggregated add;
# dense: the reference rule with dense staging (WC_OPT_SPARSE 0: non-persistent K1, 4 workgroups/CU).
for r in 1 2; do
  for v in base histA histC; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    echo "$v hist"; WCB_HIST=0.7 LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
  done
  echo "dense ref"; timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 1 0 || exit 1
  echo "sparse ref"; timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
done
