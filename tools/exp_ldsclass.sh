#!/bin/bash
# Round 6: does the 48x32x16 class (TZ 8: 40 KiB of K1 LDS, 1.6 % of C4's cells) hold the whole C4 K1
# launch at 3 workgroups/CU?  C4 with every class (WCB_C3_MASK 31) vs without the slabs (15); K1 time
# per cell should drop by ~1.6 % if not, by far more if so.  Both the reference rule and the
# global-threshold mode (whose K1 adds 16 KiB of LDS bins: 2 vs 3 workgroups/CU).
for r in 1 2; do
  for m in 31 15; do
    echo "mask $m ref"; WCB_C3_MASK=$m timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
    echo "mask $m hist"; WCB_HIST=0.7 WCB_C3_MASK=$m timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
    echo "mask $m c3rt"; WCB_C3_MASK=$m timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 20 3 3 0 || exit 1
  done
done
