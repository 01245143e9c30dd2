#!/bin/bash
# 8-wave 16K-coefficient emit tiles (61 VGPRs since the full-tile path: 4
# workgroups per CU) for smaller units: big18 = units of >= 2^18 cells (64^3),
# big15 = >= 2^15 (32^3), vs the default (>= 2^21, 128^3 only); C2, 32^3, C3
# layout (fwd only), C5, 3 reps.
S=tools/bin/wc_bench
steps=("chk18:90:LD_LIBRARY_PATH=tools/variants/big18 $S 1024 64 f64 0.999 3 1 1 1"
       "chk15:90:LD_LIBRARY_PATH=tools/variants/big15 $S 4 c3 f64 0.999 3 1 1 1")
for rep in 1 2 3; do
  for v in default big18 big15; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("ab_${v}_c2_$rep:90:$lp $S 1024 64 f64 0.999 10 2 0 0")
    steps+=("ab_${v}_s32_$rep:90:$lp $S 8192 32 f64 0.999 10 2 0 0")
    steps+=("ab_${v}_c3_$rep:90:$lp $S 4 c3 f64 0.999 10 2 0 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
