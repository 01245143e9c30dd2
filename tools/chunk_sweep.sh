#!/bin/bash
# Sweep the staged forward's emit layout and the chunked two-stream forward on
# the headline workload.  Each line: chunk_cells slots seg_max seg_min_units
# ('#' comments allowed); runs wc_bench with check=1 (payload bytes of every
# unit compared with the plain staged path's).
set -o pipefail
W="${WCB_ARGS:-1024 64 f64 0.999}"
while read -r chunk slots seg segmin _; do
    [ -z "$chunk" ] && continue
    case "$chunk" in \#*) continue ;; esac
    echo "== chunk=$chunk slots=$slots seg=$seg segmin=$segmin"
    timeout -k 5 60 tools/bin/wc_bench $W 20 3 0 0 1 0 0 1 0 0 0 "$chunk" "$slots" "$seg" "$segmin" || { echo "rc=$?"; exit 1; }
done
