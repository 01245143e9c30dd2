#!/bin/bash
# -m gpu suite, wc_bench C2 / C5 (check=1 against the conservative paths), the
# K6r order investigation (tools/gpu_rixorder.sh steps), the default bench line.
S=tools/bin/wc_bench
steps=("tests:700:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread"
       "c2:60:$S 1024 64 f64 0.999 10 2 1 1"
       "c5:90:$S 512 128 f32 0.9999 10 2 1 0"
       "bench:400:python bench.py --pmc none > gpurun_out/bench_line.txt")
A="1024 64 f64 0.999"
for x in 0 1; do
  steps+=("fetch_x$x:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/rix_x$x -o fetch -- $S $A 3 1 1 0 1 1 1 9216 4 0 $x")
  steps+=("kt_x$x:150:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rix_x$x -o kt -- $S $A 10 2 1 0 1 1 1 9216 4 0 $x")
done
for rep in 1 2; do
  steps+=("bench_x0_$rep:300:python bench.py --legs inverse --no-cpu-baseline --steps 20 --warmup 3 --pmc none > gpurun_out/bench_x0_$rep.txt")
  steps+=("bench_x1_$rep:300:python bench.py --legs inverse --no-cpu-baseline --steps 20 --warmup 3 --pmc none --rix-xcd > gpurun_out/bench_x1_$rep.txt")
done
exec tools/gpu_run.sh "${steps[@]}"
