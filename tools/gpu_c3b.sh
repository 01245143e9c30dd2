#!/bin/bash
S="tools/bin/wc_bench"
exec tools/gpu_run.sh \
 "test:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
 "c2:60:$S 1024 64 f64 0.999 20 3 1 0 1 1 1" \
 "c5:60:$S 64 128 f32 0.9999 20 3 1 0 1 1 1" \
 "c2_9999:60:$S 1024 64 f64 0.9999 20 3 1 0 1 1 1" \
 "c3kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python bench.py --workload c3 --legs inverse --no-cpu-baseline --steps 10 --warmup 2" \
 "bench:300:python bench.py --legs c3,c4,inverse --no-cpu-baseline"
