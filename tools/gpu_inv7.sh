#!/bin/bash
S="tools/bin/wc_bench"
exec tools/gpu_run.sh \
 "invtest:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "c2_check:120:$S 1024 64 f64 0.999 5 2 1 1 1 1 1" \
 "c5_check:120:$S 64 128 f32 0.9999 5 2 1 1 1 1 1" \
 "c2:60:$S 1024 64 f64 0.999 20 3 1 0 1 1 1" \
 "c5:60:$S 64 128 f32 0.9999 20 3 1 0 1 1 1" \
 "s32:60:$S 8192 32 f64 0.999 20 3 1 0 1 1 1" \
 "s16:60:$S 32768 16 f64 0.999 20 3 1 0 1 1 1" \
 "kt:120:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inv -o inv -- $S 1024 64 f64 0.999 10 2 1 0" \
 "bench:300:python bench.py"
