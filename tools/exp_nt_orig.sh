#!/bin/bash
# Round 6: nontemporal loads of the original cells in the fused-RMSE K6r (k_inverse_rows<1>, the
# C3 round trip's largest kernel, parked 75 % on those loads: r05 gpu_sq_cycles.txt); K1's cell loads
# gained 10-12 % from the same hint (gpu_nt_cells.txt).
# Prediction: C3 inverse + RMSE -3-8 %.
for r in 1 2 3 4; do
  for v in base ntorig; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    echo "$v c3"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 10 2 3 0 || exit 1
    echo "$v c3rmse2"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 10 2 2 0 || exit 1
  done
done
