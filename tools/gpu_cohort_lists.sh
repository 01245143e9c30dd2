#!/bin/bash
# Round 4: is K1 (or the emit) bound by the staging bytes?  Diagnostic cohort
# plans (timing only) with ONE item kind on all 8 XCDs and no waits: K1 tiles
# storing into a 32 / 128 MiB ring (on-die) vs the two-kernel K1; emit tiles
# reading a ring vs the two-kernel emit.  C5 shape.
S=tools/bin/wc_bench
A="512 128 f32 0.9999 10 2 0 0"
steps=("base:90:$S $A")
for v in k1list elist; do
  for sl in 1:1 4:2 16:1; do
    s=${sl%%:*}; l=${sl##*:}
    steps+=("${v}_${s}_${l}:90:LD_LIBRARY_PATH=tools/variants/$v WCB_COHORT=$s WCB_COHORT_LAG=$l $S $A")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
