# Nontemporal loads of the fused RMSE's fp64 original cells (WC_RIX_ORIG_NT, a toggle removed after this run:
# slower, profiles/r05/experiments/gpu_nt.txt); variants interleaved
for r in 1 2 3 4; do
  for v in base on; do
    L=tools/variants/$v
    echo "$v c3"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 40 5 3 0 || exit 1
    echo "$v c2r"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 40 5 3 0 || exit 1
  done
done
# K7 (wc_rmse) with cell-pair vector loads, nontemporal: k7old = the previous commit's sources
for r in 1 2 3; do
  for v in k7old k7new; do
    L=tools/variants/$v
    echo "$v c3 m7"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 30 5 7 0 || exit 1
    echo "$v c2 m7"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 30 5 7 0 || exit 1
  done
done
