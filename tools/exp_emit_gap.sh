#!/bin/bash
# Round 6: is the emit's +6 % after the nontemporal-load K1 (gpu_nt_cells.txt) K1's write-back
# draining into it?  WCB_SPLIT=us runs stage, synchronize, an idle gap of `us`, then the emit;
# variant splitsp (diagnostic only) stages sparsely at keep 0.999f in wc_forward_stage so the split
# path equals wc_forward's (the product's wc_forward_stage stages densely).
# Prediction: gap 0 = wc_forward's emit (0.206-0.22 ms at C2); gap 200-1000 us brings it to ~0.195.
for r in 1 2 3; do
  for g in none 0 200 1000; do
    for w in "1024 64 f64 0.999" "1024 64 f32 0.999"; do
      echo "gap $g $w"
      if [ $g = none ]; then timeout -k 5 60 tools/bin/wc_bench $w 10 2 0 0 || exit 1
      else WCB_SPLIT=$g LD_LIBRARY_PATH=tools/variants/splitsp timeout -k 5 60 tools/bin/wc_bench $w 10 2 0 0 || exit 1; fi
    done
  done
done
