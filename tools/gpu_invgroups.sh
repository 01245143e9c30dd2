#!/bin/bash
# Pipelined inverse (WC_OPT_INV_GROUPS) A/B after the -m gpu suite: bench.py
# inverse leg and C3 at 1 / 2 / 3 / 4 groups, alternating, twice; wc_bench C2 and
# C5 inverses at 1 and 2 groups.
S=tools/bin/wc_bench
steps=()
[ "${TESTS:-1}" = 1 ] && steps+=("tests:700:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread")
for rep in 1 2; do
  for g in 1 2 3 4; do
    steps+=("bench_g${g}_$rep:300:python bench.py --legs inverse,c3 --no-cpu-baseline --steps 20 --warmup 3 --pmc none --inv-groups $g > gpurun_out/bench_g${g}_$rep.txt")
  done
  for g in 1 2; do
    steps+=("c2_g${g}_$rep:60:$S 1024 64 f64 0.999 10 2 1 0 1 1 1 9216 4 0 0 $g")
    steps+=("c5_g${g}_$rep:90:$S 512 128 f32 0.9999 10 2 1 0 1 1 1 9216 4 0 0 $g")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
