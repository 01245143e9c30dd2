#!/bin/bash
# fp32 K1 with 16-B x-quad cell loads (default) vs the x-pair form (variant
# noquad = -DWC_K1_QUAD=0): -m gpu suite, check runs, C5 and 1024 x 64^3 fp32, 2 reps.
# (Round 3 record: the switch was removed with the measured-equal form; this script no longer builds it.)
S=tools/bin/wc_bench
steps=("tests:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
       "chk_c5:90:$S 64 128 f32 0.9999 3 1 1 1"
       "chk_f32:90:$S 256 64 f32 0.999 3 1 1 1")
for rep in 1 2; do
  for v in default noquad; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("ab_${v}_c5_$rep:90:$lp $S 512 128 f32 0.9999 10 2 0 0")
    steps+=("ab_${v}_f32_$rep:90:$lp $S 1024 64 f32 0.999 10 2 0 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
