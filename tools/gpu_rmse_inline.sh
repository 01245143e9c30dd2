#!/bin/bash
# Round 4: fused RMSE summed inside the K6r x-quad synthesis (WC_RIX_RMSE_INLINE,
# fp64 originals) vs the separate pass that re-reads the tile's output;
# C3 (4-level AMR x 4 comps, fp64) and C2 through wc_inverse_rmse (wc_bench inv
# mode 2), alternated 3 times; then the GPU tests that check the RMSE.
S=tools/bin/wc_bench
steps=()
for r in 1 2 3; do
  for v in default rmse_sep; do
    L=""; [ $v != default ] && L="LD_LIBRARY_PATH=tools/variants/$v"
    steps+=("c3_${v}_$r:90:$L $S 4 c3 f64 0.999 10 2 2 0")
    steps+=("c2_${v}_$r:90:$L $S 1024 64 f64 0.999 10 2 2 0")
  done
done
steps+=("tests:400:python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread")
exec tools/gpu_run.sh "${steps[@]}"
