#!/bin/bash
# K6r tile order A/B: XCD-grouped (default) vs unit order (rixnat).
S="tools/bin/wc_bench"
steps=("tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
for v in default rixnat default rixnat; do
  if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
  steps+=("r_${v}_c2chk:60:$lp $S 1024 64 f64 0.999 5 2 1 1 1 1 1")
  steps+=("r_${v}_c2:60:$lp $S 1024 64 f64 0.999 20 3 1 0 1 1 1")
  steps+=("r_${v}_c5:60:$lp $S 64 128 f32 0.9999 20 3 1 0 1 1 1")
  steps+=("r_${v}_s32:60:$lp $S 8192 32 f64 0.999 20 3 1 0 1 1 1")
  steps+=("r_${v}_s16:60:$lp $S 32768 16 f64 0.999 20 3 1 0 1 1 1")
done
exec tools/gpu_run.sh "${steps[@]}"
