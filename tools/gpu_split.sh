#!/bin/bash
S="tools/bin/wc_bench"
steps=()
for cfg in "1024 64 f64 0.999" "64 128 f32 0.9999" "8192 32 f64 0.999" "32768 16 f64 0.999"; do
  set -- $cfg; n="$1_$2"
  steps+=("s0_$n:60:$S $cfg 20 3 0 0 1 1 1 9216 4 0 0")
  steps+=("s1_$n:60:$S $cfg 20 3 0 0 1 1 1 9216 4 0 1")
done
exec tools/gpu_run.sh \
 "test:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread" \
 "c2_check:120:$S 1024 64 f64 0.999 5 2 1 1 1 1 1 9216 4 0 1" \
 "${steps[@]}"
