#!/bin/bash
# K6r x-quad stores and blocked tile order (A/B against the float2 build in tools/variants/f2).
S="tools/bin/wc_bench"
steps=()
for cfg in "1024 64 f64 0.999" "64 128 f32 0.9999" "8192 32 f64 0.999" "32768 16 f64 0.999"; do
  set -- $cfg; n="$1_$2"
  for b in 1 0; do
    steps+=("q${b}_$n:60:$S $cfg 20 3 1 0 1 1 1 9216 4 $b")
    steps+=("f2${b}_$n:60:LD_LIBRARY_PATH=tools/variants/f2 $S $cfg 20 3 1 0 1 1 1 9216 4 $b")
  done
done
exec tools/gpu_run.sh \
 "invtest:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "c2_check:120:$S 1024 64 f64 0.999 5 2 1 1 1 1 1" \
 "${steps[@]}"
