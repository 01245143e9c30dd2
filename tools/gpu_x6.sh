#!/bin/bash
# Transform tiles of 64 x 1 x 16 blocks for units with >= 64 x-blocks (x6 =
# -DWC_TILE_X=6: whole 512-B fp32 rows of a 128^3 unit, two adjacent rows = 1 KB
# per z plane, 16-coefficient segments) vs 32 x 1 x 32 (default); check runs
# against the conservative path, then C5 and 128^3 fp64, 2 reps.
# (Round 3 record: WC_TILE_X was removed after the form measured slower; this script no longer builds it.)
S=tools/bin/wc_bench
steps=("chk_x6:90:LD_LIBRARY_PATH=tools/variants/x6 $S 64 128 f32 0.9999 3 1 1 1"
       "chk_x6_f64:90:LD_LIBRARY_PATH=tools/variants/x6 $S 32 128 f64 0.999 3 1 1 1")
for rep in 1 2; do
  for v in default x6; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("ab_${v}_c5_$rep:90:$lp $S 512 128 f32 0.9999 10 2 0 0")
    steps+=("ab_${v}_f64128_$rep:90:$lp $S 256 128 f64 0.999 10 2 0 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
