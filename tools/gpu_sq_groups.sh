#!/bin/bash
# SQ cycle breakdown (tools/sq_summary.py) and HBM bytes of K1 / the emit per C4 unit class
# (WCB_C3_MASK: 2 = the L1 64^3 units, 4 = the L2 32^3 units, 8 = the L3 16^3 units), forward only.
# Question (gpu_c4_groups.txt): why is the 32^3 K1 40 % slower per cell than the 64^3 one?
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
steps=()
for m in 2 4 8; do
  steps+=("sq_m$m:90:WCB_C3_MASK=$m timeout -s KILL 80 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sqg -o m$m -- tools/bin/wc_bench 80 c3 f64 0.999 3 1 0 0")
  steps+=("fe_m$m:90:WCB_C3_MASK=$m timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/sqg -o fm$m -- tools/bin/wc_bench 80 c3 f64 0.999 3 1 0 0")
  steps+=("wr_m$m:90:WCB_C3_MASK=$m timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/sqg -o wm$m -- tools/bin/wc_bench 80 c3 f64 0.999 3 1 0 0")
done
steps+=("sq_sum:30:python tools/sq_summary.py gpurun_out/sqg/m2_counter_collection.csv gpurun_out/sqg/m4_counter_collection.csv gpurun_out/sqg/m8_counter_collection.csv > gpurun_out/sqg_summary.txt")
exec tools/gpu_run.sh "${steps[@]}"
