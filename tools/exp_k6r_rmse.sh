# fused fp64 RMSE (K6r OT=1): prefetch slots given up (WC_RIX_RMSE_ROUNDS_LESS)
for v in l3 l5 l7 l9 l11; do
  L=tools/variants/$v
  for r in 1 2; do
    echo "$v c3 mode3"; LD_LIBRARY_PATH=$L tools/bin/wc_bench 4 c3 f64 0.999 20 3 3 0
    echo "$v c2 mode3"; LD_LIBRARY_PATH=$L tools/bin/wc_bench 1024 64 f64 0.999 20 3 3 0
  done
done
