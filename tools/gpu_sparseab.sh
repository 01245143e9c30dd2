#!/bin/bash
# Sparse vs dense coefficient staging (wc_bench argument 10) on C5 and C2.
S="tools/bin/wc_bench"
steps=()
for rep in 1 2; do
  for sp in 1 0; do
    steps+=("ab_sp${sp}_c5full_$rep:60:$S 512 128 f32 0.9999 10 2 0 0 1 $sp 1")
    steps+=("ab_sp${sp}_c5_$rep:60:$S 64 128 f32 0.9999 20 3 0 0 1 $sp 1")
    steps+=("ab_sp${sp}_c2_$rep:60:$S 1024 64 f64 0.999 20 3 0 0 1 $sp 1")
    steps+=("ab_sp${sp}_f32c2_$rep:60:$S 1024 64 f32 0.999 20 3 0 0 1 $sp 1")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
