#!/bin/bash
# Round 4: where the cohort forward's time goes (diagnostic variants of
# tools/build_variants.sh, timing only): no waits, plain ring accesses, one item
# kind only, no emit look-back; C5 at two cohort shapes.
S=tools/bin/wc_bench
A="512 128 f32 0.9999 10 2 0 0"
steps=()
for sl in ${COHORTS:-4:2 1:1}; do
  s=${sl%%:*}; l=${sl##*:}
  steps+=("coh${s}_${l}_default:90:WCB_COHORT=$s WCB_COHORT_LAG=$l $S $A")
  for v in ${VARIANTS:-nowait plain k1only eonly nolb}; do
    steps+=("coh${s}_${l}_$v:90:LD_LIBRARY_PATH=tools/variants/$v WCB_COHORT=$s WCB_COHORT_LAG=$l $S $A")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
