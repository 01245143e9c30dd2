#!/bin/bash
# Emit blocks of 2 tiles (default, MINB 4 with spills), MINB 3 / 2, and 1 / 4 tiles per block.
S="tools/bin/wc_bench"
steps=()
for cfg in "1024 64 f64 0.999" "64 128 f32 0.9999" "8192 32 f64 0.999" "32768 16 f64 0.999"; do
  set -- $cfg; n="$1_$2"
  for v in default m3 m2 nt1 nt4; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("${v}_$n:60:$lp $S $cfg 20 3 0 0 1 1 1")
  done
done
exec tools/gpu_run.sh \
 "test:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "c2_check:120:$S 1024 64 f64 0.999 5 2 1 1 1 1 1" \
 "${steps[@]}"
