#!/bin/bash
# K1 specialised for the 32 x 1 x 32 tile shape (default) vs the generic body
# (nos32 = -DWC_K1_S32=0): -m gpu suite, check runs against the conservative
# path, then C2, C5 and 1024 x 64^3 fp32, 2 reps.
S=tools/bin/wc_bench
steps=("tests:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
       "chk_c2:90:$S 1024 64 f64 0.999 3 1 1 1"
       "chk_c5:90:$S 64 128 f32 0.9999 3 1 1 1")
for rep in $(seq 1 ${REPS:-2}); do
  for v in default ${VARIANTS:-nos32}; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("ab_${v}_c2_$rep:90:$lp $S 1024 64 f64 0.999 10 2 0 0")
    steps+=("ab_${v}_c5_$rep:90:$lp $S 512 128 f32 0.9999 10 2 0 0")
    steps+=("ab_${v}_f32_$rep:90:$lp $S 1024 64 f32 0.999 10 2 0 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
