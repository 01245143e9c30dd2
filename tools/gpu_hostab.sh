#!/bin/bash
# wc_forward_host A/B (bench.py host leg, PCIe-inclusive C2) after the -m gpu suite.
steps=("tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then lp=""; else lp="WCAMD_LIB=tools/variants/$v/libwavelet_amd.so"; fi
    steps+=("hostab_${v}_$rep:180:$lp python bench.py --legs host --no-cpu-baseline --steps 5 --warmup 2 --leg-steps 5")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
