#!/bin/bash
# Where the waves of each kernel spend their cycles (round 3): SQ_WAVE_CYCLES =
# SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (issue stall)
# + SQ_ACTIVE_INST_ANY, plus LDS bank-conflict cycles; C2 (forward + inverse)
# and C5 (forward), one --pmc pass each.
S=tools/bin/wc_bench
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
exec tools/gpu_run.sh \
 "sq_c2:90:timeout -s KILL 80 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq3 -o c2 -- $S 1024 64 f64 0.999 3 1 1 0" \
 "sq_c5:90:timeout -s KILL 80 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq3 -o c5 -- $S 512 128 f32 0.9999 3 1 0 0"
