#!/bin/bash
S="tools/bin/wc_bench"
steps=()
for rep in 1 2; do
  for v in default rix21; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("ab_${v}_c2_$rep:60:$lp $S 1024 64 f64 0.999 20 3 1 0 1 1 1")
  done
done
steps+=("ab_rix21_c2chk:60:LD_LIBRARY_PATH=tools/variants/rix21 $S 1024 64 f64 0.999 5 2 1 1 1 1 1")
exec tools/gpu_run.sh "${steps[@]}"
