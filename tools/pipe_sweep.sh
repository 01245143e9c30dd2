#!/bin/bash
# Sweep the pipelined forward kernel's tuning options on the headline workload.
# Each line: lag ring claim prefetch wgs ; runs wc_bench with stats on.
set -o pipefail
W="${WCB_ARGS:-1024 64 f64 0.999}"
mkdir -p gpurun_out
while read -r lag ring claim pf wgs; do
    [ -z "$lag" ] && continue
    echo "== lag=$lag ring=$ring claim=$claim prefetch=$pf wgs=$wgs"
    timeout -k 5 60 tools/bin/wc_bench $W 10 2 0 1 0 $lag $ring $claim $pf $wgs 1 || { echo "rc=$?"; exit 1; }
done
