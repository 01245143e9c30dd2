#!/bin/bash
# Kernel trace of the C3 layout: forward (headline of --workload c3) and its inverse leg.
exec tools/gpu_run.sh \
 "c3kt:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python bench.py --workload c3 --legs inverse --no-cpu-baseline --steps 10 --warmup 2"
