#!/bin/bash
# Round 4: where the row index (K5) spends its time.  Diagnostic builds (timing
# only, results invalid): rnolb = no look-back, rnorows = no row-entry writes,
# rnoload = synthetic runs instead of the payload loads (-DWC_XP_RIX_NOLOAD: a
# temporary patch of k_rowindex's run load, `v[r] = k < n ? (k & 7u) : 0u`,
# not kept in the sources); rbase = the default sources built the same way.  C2 and C5 inverse, alternated 3 times.
S=tools/bin/wc_bench
steps=()
for r in 1 2 3; do
  for v in rbase rnolb rnorows rnoload; do
    L="LD_LIBRARY_PATH=tools/variants/$v"
    steps+=("x2_${v}_$r:90:$L $S 1024 64 f64 0.999 10 2 1 0")
    steps+=("x5_${v}_$r:90:$L $S 512 128 f32 0.9999 10 2 1 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
