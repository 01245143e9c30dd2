#!/bin/bash
# Diagnostic variants: row index (no look-back / no row writes) and emit (no look-back / no pair stores).
S="tools/bin/wc_bench"
steps=()
for v in default nolb norows nolbrows enolb enostore; do
  if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
  steps+=("x_${v}_c2:60:$lp $S 1024 64 f64 0.999 20 3 1 0 1 1 1")
  steps+=("x_${v}_c5:60:$lp $S 64 128 f32 0.9999 20 3 1 0 1 1 1")
done
exec tools/gpu_run.sh "${steps[@]}"
