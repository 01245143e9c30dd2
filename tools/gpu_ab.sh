#!/bin/bash
# Generic A/B of libwavelet_amd.so variants (tools/build_variants.sh) on wc_bench:
#   VARIANTS='a b'  variants besides the default build, REPS (2), INV (0 forward
#   only, 1 + inverse, 2 + fused inverse/RMSE), TESTS=1 runs -m gpu first,
#   SHAPES (default 'c2 c5 f32').  tools/ab_report.py gpurun_out summarises.
S=tools/bin/wc_bench
declare -A ARGS=([c2]="1024 64 f64 0.999" [c5]="512 128 f32 0.9999" [f32]="1024 64 f32 0.999" [s32]="4096 32 f64 0.999" [s16]="16384 16 f64 0.999")
steps=()
[ "${TESTS:-0}" = 1 ] && steps+=("tests:400:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread")
steps+=("chk_c2:90:$S 1024 64 f64 0.999 3 1 ${INV:-0} 1" "chk_c5:90:$S 64 128 f32 0.9999 3 1 ${INV:-0} 1")
for rep in $(seq 1 ${REPS:-2}); do
  for v in default ${VARIANTS}; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    for s in ${SHAPES:-c2 c5 f32}; do
      steps+=("ab_${v}_${s}_$rep:90:$lp $S ${ARGS[$s]} 10 2 ${INV:-0} 0")
    done
  done
done
exec tools/gpu_run.sh "${steps[@]}"
