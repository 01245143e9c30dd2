#!/bin/bash
# Profiles of the headline workload (1024 x 64^3 fp64, keep 0.999f) for profiles/.
# Run on the GPU box through tools/gpu_run.sh; every step has its own limit.
#   kt_bench   rocprofv3 kernel trace + stats of bench.py itself
#   kt_wcb     the same workload through the torch-free C++ driver
#   pmc_fetch  FETCH_SIZE per dispatch   (separate pass: FETCH costs 3 TCC slots)
#   pmc_write  WRITE_SIZE per dispatch
# then: python tools/pmc_summary.py gpurun_out/prof_wcb/wcb_kernel_stats.csv \
#         --fetch gpurun_out/prof_fetch/fetch_counter_collection.csv \
#         --write gpurun_out/prof_write/write_counter_collection.csv --out profiles/<round>/summary.json
set -o pipefail
W="${WCB_ARGS:-1024 64 f64 0.999}"
F="${WCB_PIPE:-0}"    # 0: the default staged kernels, 1: the pipelined kernel
exec tools/gpu_run.sh \
  "kt_bench:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline" \
  "kt_wcb:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wcb -o wcb -- tools/bin/wc_bench $W 10 2 1 $F" \
  "pmc_fetch:200:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- tools/bin/wc_bench $W 3 1 1 $F" \
  "pmc_write:200:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- tools/bin/wc_bench $W 3 1 1 $F"
