#!/bin/bash
S="tools/bin/wc_bench"
exec tools/gpu_run.sh \
 "test:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "c2_check:120:$S 1024 64 f64 0.999 5 2 1 1 1 1 1" \
 "c2:60:$S 1024 64 f64 0.999 20 3 1 0 1 1 1" \
 "c2t:60:$S 1024 64 f64 0.999 20 3 1 0 0 1 1" \
 "c5:60:$S 64 128 f32 0.9999 20 3 1 0 1 1 1" \
 "s32:60:$S 8192 32 f64 0.999 20 3 1 0 1 1 1" \
 "s16:60:$S 32768 16 f64 0.999 20 3 1 0 1 1 1" \
 "bench:300:python bench.py --legs inverse --no-cpu-baseline"
