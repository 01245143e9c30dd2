#!/bin/bash
# Round 4: the cohort forward (WC_OPT_COHORT) — GPU parity tests, then C5
# (512 x 128^3 fp32, keep 0.9999f) timed by wc_bench at several cohort sizes
# and lags beside the staged two-kernel path, and a full-batch check against
# the conservative path (tickets, dense staging, no cohort).
S=tools/bin/wc_bench
steps=("tests:300:python -u -m pytest tests/test_gpu_cohort.py -x -v --timeout 120 --timeout-method thread")
steps+=("c5_base:90:$S 512 128 f32 0.9999 10 2 0 0")
for sl in ${COHORTS:-1:1 2:1 2:2 4:1 4:2 8:1}; do
  s=${sl%%:*}; l=${sl##*:}
  steps+=("c5_coh${s}_${l}:90:WCB_COHORT=$s WCB_COHORT_LAG=$l $S 512 128 f32 0.9999 10 2 0 0")
done
steps+=("c5_check:120:WCB_COHORT=${CHECK_S:-2} WCB_COHORT_LAG=${CHECK_L:-2} $S 512 128 f32 0.9999 3 1 0 1")
[ -n "$EXTRA" ] && steps+=($EXTRA)
exec tools/gpu_run.sh "${steps[@]}"
