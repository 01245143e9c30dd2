#!/bin/bash
# SQ counters of the forward and inverse kernels on C2 (one --pmc pass each, own time limit)
W="1024 64 f64 0.999 3 1 1"
exec tools/gpu_run.sh \
 "sqc:90:timeout -s KILL 80 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CU_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/sqc -o sqc -- tools/bin/wc_bench $W"
