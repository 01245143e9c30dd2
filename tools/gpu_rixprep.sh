#!/bin/bash
# Round 4: the row index's record pass (WC_OPT_RIX_PREP): k_rix_prep reads each
# pair tile's unit offset and header once and writes a 32-B record, so a K5
# block's run loads wait on one record load instead of tile -> offset ->
# header (2 dependent round trips fewer; blocks past a payload exit after one).
# Predicted (the emit's block descriptor removed one round trip: -7 %): K5
# -10..15 % at C2/C5 net of the record pass (~3-5 us); inverse -3..5 %.
# (Record: measured no change and removed; this script no longer builds it.)
S=tools/bin/wc_bench
steps=("tests:400:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -x -q --timeout 200 --timeout-method thread -k 'inverse or rle or malformed or sparse_decode or c5'")
for r in 1 2 3; do
  for v in 0 1; do
    steps+=("p2_${v}_$r:90:WCB_RIX_PREP=$v $S 1024 64 f64 0.999 10 2 1 0")
    steps+=("p5_${v}_$r:90:WCB_RIX_PREP=$v $S 512 128 f32 0.9999 10 2 1 0")
    steps+=("p3_${v}_$r:90:WCB_RIX_PREP=$v $S 4 c3 f64 0.999 10 2 2 0")
  done
done
exec tools/gpu_run.sh "${steps[@]}"
