#!/bin/bash
# C3 round-trip A/B of library variants through bench.py (WCAMD_LIB), after
# the -m gpu suite.  usage: tools/gpu_c3ab.sh variant...   ("default" = in-tree lib)
steps=("tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then lp=""; else lp="WCAMD_LIB=tools/variants/$v/libwavelet_amd.so"; fi
    steps+=("c3ab_${v}_$rep:120:$lp python bench.py --legs c3 --no-cpu-baseline --steps 5 --warmup 2 --leg-steps 10")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
