#!/bin/bash
# Round 6: the drop-in write-behind loop, this round's queue (per-file flush, never destroyed,
# atexit drain, flushers woken only when one waits) vs round 5's (tools/variants/wbold), four timed
# passes per process (DROPIN_WB_REPS), two processes each, in ABBA order.
for r in 1 2; do
  order="base wbold"; [ $r = 2 ] && order="wbold base"  # ABBA: the box's drift cancels
  for v in $order; do
    L=wavelet-compression_amd/lib; [ $v = wbold ] && L=tools/variants/wbold
    echo "$v"; DROPIN_WB_REPS=4 LD_LIBRARY_PATH=$L timeout -k 5 300 tools/bin/dropin_bench /tmp/wcamd_dropin_ab_$$ 4 0.999 || exit 1
  done
done
