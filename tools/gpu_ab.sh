#!/bin/bash
# A/B of library variants (tools/variants/<name>/, "default" = the in-tree lib)
# over the wc_bench shapes, after the -m gpu suite; optional PMC passes.
# usage: tools/gpu_ab.sh [--no-tests] [--pmc COUNTER] variant...
S="tools/bin/wc_bench"
tests=1; pmc=""
while [ $# -gt 0 ]; do
  case "$1" in
    --no-tests) tests=0; shift;;
    --pmc) pmc="$2"; shift 2;;
    *) break;;
  esac
done
steps=()
[ $tests = 1 ] && steps+=("tests:300:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
for rep in 1 2; do
  for v in "$@"; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    [ $rep = 1 ] && steps+=("ab_${v}_c2chk:60:$lp $S 1024 64 f64 0.999 5 2 1 1 1 1 1")
    steps+=("ab_${v}_c2_$rep:60:$lp $S 1024 64 f64 0.999 20 3 1 0 1 1 1")
    steps+=("ab_${v}_c5_$rep:60:$lp $S 64 128 f32 0.9999 20 3 1 0 1 1 1")
    steps+=("ab_${v}_s32_$rep:60:$lp $S 8192 32 f64 0.999 20 3 1 0 1 1 1")
    steps+=("ab_${v}_s16_$rep:60:$lp $S 32768 16 f64 0.999 20 3 1 0 1 1 1")
  done
done
if [ -n "$pmc" ]; then
  for v in "$@"; do
    if [ $v = default ]; then lp=""; else lp="LD_LIBRARY_PATH=tools/variants/$v"; fi
    steps+=("pmc_${v}:90:$lp rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/pmc_ab -o $v -- $S 1024 64 f64 0.999 3 1 1 0 1 1 1")
  done
fi
exec tools/gpu_run.sh "${steps[@]}"
