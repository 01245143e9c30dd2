#!/bin/bash
# Row-index tile 8192 vs 4096 pairs (tools/variants/t4k), x-quad K6r.
S="tools/bin/wc_bench"
steps=()
for cfg in "1024 64 f64 0.999" "64 128 f32 0.9999" "8192 32 f64 0.999" "32768 16 f64 0.999"; do
  set -- $cfg; n="$1_$2"
  steps+=("t8k_$n:60:$S $cfg 20 3 1 0 1 1 1")
  steps+=("t4k_$n:60:LD_LIBRARY_PATH=tools/variants/t4k $S $cfg 20 3 1 0 1 1 1")
done
exec tools/gpu_run.sh \
 "invtest:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "c2_check:120:$S 1024 64 f64 0.999 5 2 1 1 1 1 1" \
 "c5_check:120:$S 64 128 f32 0.9999 5 2 1 1 1 1 1" \
 "${steps[@]}" \
 "bench:300:python bench.py --legs inverse,c3 --no-cpu-baseline"
