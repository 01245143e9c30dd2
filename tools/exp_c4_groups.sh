#!/bin/bash
# Round 6: where the C4 emit's lower byte rate lives (C4 emit 26.8 GB of counter traffic in 6.29 ms
# = 4.3 TB/s vs C2's 4.9).  WCB_C3_MASK runs one unit group of the C4 batch at a time (bit 0 L0
# 64^3, 1 L1 64^3, 2 L2 32^3, 3 L3 16^3 cubes, 4 the 48x32x16 slabs); forward only, 10 steps.
# Prediction: the 64^3 groups run their emit at C2's per-byte rate; the 16^3 / 32^3 groups (one or
# four emit tiles per unit, half-full tiles at 16^3) hold the lower rate.
for r in 1 2; do
  for m in 31 1 2 4 8 16 3 28; do
    echo "mask $m"; WCB_C3_MASK=$m timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
  done
done
