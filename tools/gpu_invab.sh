#!/bin/bash
steps=()
for rep in 1 2 3; do
  for v in default rixnat; do
    if [ $v = default ]; then lp=""; else lp="WCAMD_LIB=tools/variants/$v/libwavelet_amd.so"; fi
    steps+=("invab_${v}_$rep:120:$lp python bench.py --legs inverse --no-cpu-baseline --steps 20 --warmup 3")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
