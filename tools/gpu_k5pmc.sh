#!/bin/bash
# Round 4: texture-path and read-latency counters of every kernel of the C2
# forward + inverse (wc_bench), to see what the row index (K5) waits on.
# Predicted: if K5's run loads (64 per-lane 4-B addresses per instruction) are
# address-bound, TA busy near 100 % during K5; if latency-bound, a high
# TCP->TCC read latency.
S=tools/bin/wc_bench
o=gpurun_out/pmc_k5
exec tools/gpu_run.sh \
  "k5_ta:120:timeout -s KILL 100 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d $o -o ta -- $S 1024 64 f64 0.999 3 1 1 0" \
  "k5_tcp:120:timeout -s KILL 100 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --output-format csv -d $o -o tcp -- $S 1024 64 f64 0.999 3 1 1 0"
