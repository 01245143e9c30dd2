#!/bin/bash
# Round 4: the row index without its look-back and second barrier (variant fakelb
# = -DWC_XP_RIX_FAKELB, a temporary patch of k_rowindex, not kept: a made-up
# prefix t x 13312 positions, timing only) vs the same sources built alike.
S=tools/bin/wc_bench
steps=()
for r in 1 2 3; do
  for v in fbase fakelb; do
    L="LD_LIBRARY_PATH=tools/variants/$v"
    steps+=("f2_${v}_$r:90:$L $S 1024 64 f64 0.999 10 2 1 0")
    steps+=("f5_${v}_$r:90:$L $S 512 128 f32 0.9999 10 2 1 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
