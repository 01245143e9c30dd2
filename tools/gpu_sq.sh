#!/bin/bash
# SQ cycle breakdown (tools/sq_summary.py: parked / issue-stalled / issuing shares of the wave
# cycles, LDS conflicts) of the forward and inverse kernels: C2 (wc_forward + wc_inverse) and C3
# (the round trip: wc_forward_rows + wc_inverse_rows with the fused RMSE).  One --pmc pass per
# workload (8 SQ counters), each under its own time limit.
C="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
exec tools/gpu_run.sh \
 "sq_c2:90:timeout -s KILL 80 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq5 -o c2 -- tools/bin/wc_bench 1024 64 f64 0.999 3 1 1 0" \
 "sq_c3:90:timeout -s KILL 80 rocprofv3 --pmc $C --output-format csv -d gpurun_out/sq5 -o c3 -- tools/bin/wc_bench 4 c3 f64 0.999 3 1 3 0" \
 "sq_sum:30:python tools/sq_summary.py gpurun_out/sq5/c2_counter_collection.csv gpurun_out/sq5/c3_counter_collection.csv > gpurun_out/sq5_summary.txt"
