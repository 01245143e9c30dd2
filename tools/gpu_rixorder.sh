#!/bin/bash
# K6r tile order: unit order (default) vs XCD-grouped (WC_OPT_RIX_XCD), the
# round-2 contradiction (fewer fetched bytes, slower through bench.py): one
# FETCH_SIZE pass and one kernel trace of each order through wc_bench, then
# bench.py's inverse leg in both orders, alternating, twice.
S=tools/bin/wc_bench
A="1024 64 f64 0.999"
steps=()
for x in 0 1; do
  steps+=("fetch_x$x:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/rix_x$x -o fetch -- $S $A 3 1 1 0 1 1 1 9216 4 0 $x")
  steps+=("kt_x$x:150:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rix_x$x -o kt -- $S $A 10 2 1 0 1 1 1 9216 4 0 $x")
done
for rep in 1 2; do
  steps+=("bench_x0_$rep:300:python bench.py --legs inverse --no-cpu-baseline --steps 20 --warmup 3 --pmc none > gpurun_out/bench_x0_$rep.txt")
  steps+=("bench_x1_$rep:300:python bench.py --legs inverse --no-cpu-baseline --steps 20 --warmup 3 --pmc none --rix-xcd > gpurun_out/bench_x1_$rep.txt")
done
exec tools/gpu_run.sh "${steps[@]}"
