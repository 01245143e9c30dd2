#!/bin/bash
# Round 4: K6r range-major rounds (WC_RIX_RANGEMAJOR 1: prefetch slot = range,
# round fields from immediate-lane readlanes) vs flat round order (per-round
# ballot + popcount + readlanes); C2 and C5 wc_inverse, C3 wc_inverse_rmse,
# alternated 3 times; then the -m gpu suite.
S=tools/bin/wc_bench
steps=()
for r in 1 2 3; do
  for v in default flat; do
    L=""; [ $v != default ] && L="LD_LIBRARY_PATH=tools/variants/$v"
    steps+=("c2_${v}_$r:90:$L $S 1024 64 f64 0.999 10 2 1 0")
    steps+=("c5_${v}_$r:90:$L $S 512 128 f32 0.9999 10 2 1 0")
    steps+=("c3_${v}_$r:90:$L $S 4 c3 f64 0.999 10 2 2 0")
  done
done
for r in 1 2; do
  for v in default spec2; do
    L=""; [ $v != default ] && L="LD_LIBRARY_PATH=tools/variants/$v"
    steps+=("c5f_${v}_$r:90:$L $S 512 128 f32 0.9999 10 2 0 0")
  done
done
steps+=("tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread")
exec tools/gpu_run.sh "${steps[@]}"
