#!/bin/bash
# Round 4: is the row index's compute issue-bound?  Variant fastscan =
# -DWC_XP_RIX_FASTSCAN (a temporary patch of k_rowindex, not kept): the
# non-saturating fused-DPP wave scan instead of the saturating one (mov_dpp +
# add-with-clamp per step), same sums for these payloads.
# Predicted: if K5's non-load time is instruction issue, K5 -5..15 %; else =.
S=tools/bin/wc_bench
steps=()
for r in 1 2 3; do
  for v in sbase fastscan; do
    L="LD_LIBRARY_PATH=tools/variants/$v"
    steps+=("s2_${v}_$r:90:$L $S 1024 64 f64 0.999 10 2 1 0")
    steps+=("s5_${v}_$r:90:$L $S 512 128 f32 0.9999 10 2 1 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
