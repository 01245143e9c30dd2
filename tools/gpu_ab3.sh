#!/bin/bash
# Round-3 A/B: K6r pair-count clamp (default vs -DWC_RIX_CLAMP=0), packed rows
# for D = 128 (WC_OPT_SPARSE 2 vs 1) on C5 shapes, after the -m gpu suite.
# wc_bench args: boxes dim dtype keep steps warmup inverse check ordered sparse rows rix_lds rix_tx rix_blocked k1_xcd rix_xcd
S="tools/bin/wc_bench"
steps=()
[ "${TESTS:-1}" = 1 ] && steps+=("tests:700:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread")
steps+=("chk_c5pk:60:$S 64 128 f32 0.9999 3 1 1 1 1 2 1 9216 4 0 0 0")
for rep in 1 2; do
  for v in default noclamp; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("inv_${v}_$rep:60:$lp $S 1024 64 f64 0.999 10 2 1 0 1 1 1 9216 4 0 0 0")
  done
  steps+=("inv_rixxcd_$rep:60:$S 1024 64 f64 0.999 10 2 1 0 1 1 1 9216 4 0 0 1")
  for sp in 1 2; do
    steps+=("c5_s${sp}_$rep:90:$S 512 128 f32 0.9999 10 2 0 0 1 $sp 1 9216 4 0 0 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
