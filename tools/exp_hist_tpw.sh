#!/bin/bash
# Round 6: the global-threshold K1 (k_transform_hist, plain LDS bin adds) with its tiles per workgroup:
# base = persistent (resident grid, one flush of the LDS bins per workgroup); tpwN = ceil(tiles / N)
# workgroups, N tiles each (one flush per N tiles: ~N times fewer 64-bit bin atomics than N = 1).
# Prediction: tpw1 loses to the flush atomics (~469k tiles x ~60 nonzero bins at C4), tpw4 / tpw16
# recover the dispatcher's balance at a fraction of them and beat the persistent form by ~0.3-0.5 ms.
for r in 1 2 3; do
  for v in base ${TPW_SET:-tpw1 tpw4 tpw16}; do
    L=tools/variants/$v; [ $v = base ] && L=wavelet-compression_amd/lib
    echo "$v c4hist"; WCB_HIST=0.7 LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
  done
  echo "base c4ref"; timeout -k 5 60 tools/bin/wc_bench 80 c3 f64 0.999 10 2 0 0 || exit 1
done
