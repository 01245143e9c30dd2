#!/bin/bash
# Round 4: the pipelined inverse (WC_OPT_INV_GROUPS: row index of group g + 1
# beside K6r of group g) with K6r's persistent grid at 4/4 (gbase), 3/4 (g3) or
# 2/4 (g2) of the resident capacity (diagnostic -DWC_XP_K6R_GRID_NUM, a
# temporary patch of persistent_grid), so the latency-bound row index finds
# free slots beside the streaming K6r.  Predicted: if the two overlap, the
# C2 inverse falls toward its 2.76 GB / 6.2 TB/s = 0.45 ms floor (-10 %);
# with a full K6r grid (gbase) groups measured slower (0.62 vs 0.53 ms, round 3).
S=tools/bin/wc_bench
steps=()
for rep in 1 2; do
  for v in gbase g3 g2; do
    for g in 1 2 4; do
      L="LD_LIBRARY_PATH=tools/variants/$v"
      steps+=("k2_${v}_g${g}_$rep:60:$L $S 1024 64 f64 0.999 10 2 1 0 1 1 1 9216 4 0 0 $g")
      steps+=("k5_${v}_g${g}_$rep:90:$L $S 512 128 f32 0.9999 10 2 1 0 1 1 1 9216 4 0 0 $g")
    done
  done
done
exec tools/gpu_run.sh "${steps[@]}"
