#!/bin/bash
# Round 4: what the row index's blocks past each payload's pairs cost (the plan
# launches ncoeff / 4096 + 1 tiles per unit; C2 needs ~20 of 65, C5 ~230 of
# 513).  Diagnostic build capping the plan at the tiles a kept fraction of
# 0.47 needs (timing only, valid for these payloads), alternated 3 times.
S=tools/bin/wc_bench
steps=()
for r in 1 2 3; do
  for v in default cap; do
    L=""; [ $v != default ] && L="LD_LIBRARY_PATH=tools/variants/$v"
    steps+=("rc2_${v}_$r:90:$L $S 1024 64 f64 0.999 10 2 1 0")
    steps+=("rc5_${v}_$r:90:$L $S 512 128 f32 0.9999 10 2 1 0")
  done
done
steps+=("tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread")
exec tools/gpu_run.sh "${steps[@]}"
