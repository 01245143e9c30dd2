#!/bin/bash
# Packed-row staging A/B (WC_OPT_SPARSE 2 vs 1) and the XCD-grouped transform
# order (WC_OPT_K1_XCD 1 vs 0) through wc_bench, after the -m gpu suite.
# wc_bench args: boxes dim dtype keep steps warmup inverse check ordered sparse rows rix_lds rix_tx rix_blocked k1_xcd
S="tools/bin/wc_bench"
steps=()
[ "${TESTS:-1}" = 1 ] && steps+=("tests:700:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread")
steps+=("chk_c2:60:$S 1024 64 f64 0.999 3 1 1 1 1 2 1 9216 4 0 1")
steps+=("chk_c5:60:$S 64 128 f32 0.9999 3 1 1 1 1 2 1 9216 4 0 1")
for rep in 1 2; do
  for cfg in "2 1" "1 1" "2 0" "1 0"; do
    set -- $cfg
    steps+=("c2_s$1x$2_$rep:60:$S 1024 64 f64 0.999 20 3 1 0 1 $1 1 9216 4 0 $2")
    steps+=("c5_s$1x$2_$rep:60:$S 64 128 f32 0.9999 20 3 0 0 1 $1 1 9216 4 0 $2")
    steps+=("f32_s$1x$2_$rep:60:$S 1024 64 f32 0.999 20 3 0 0 1 $1 1 9216 4 0 $2")
  done
done
[ "${BENCH:-1}" = 1 ] && steps+=("bench:400:python bench.py > gpurun_out/bench_line.txt")
exec tools/gpu_run.sh "${steps[@]}"
