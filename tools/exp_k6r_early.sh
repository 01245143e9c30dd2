# (WC_RIX_ORIG_EARLY was a patch of wc_inverse.hip, reverted after this run: gpu_k6r_early.txt)
# fused fp64 RMSE (K6r OT=1): original cells issued before the scatter (WC_RIX_ORIG_EARLY),
# against the slots they cost (WC_RIX_RMSE_ROUNDS_LESS) and a 3-wave register budget (WC_RIX_MINW)
for v in base e1l13 e0l13 e2m3 e2m3l3 e0m3l3; do
  L=tools/variants/$v
  for r in 1 2; do
    echo "$v c3 mode3"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 20 3 3 0 || exit 1
    echo "$v c2 mode3"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 20 3 3 0 || exit 1
  done
done
