#!/bin/bash
# SQ counters of the inverse kernels (one --pmc pass each, own time limit)
W="1024 64 f64 0.999 3 1 1 1 1 1 1"
exec tools/gpu_run.sh \
 "list:60:rocprofv3 -L > gpurun_out/counters_list.txt 2>&1" \
 "sq1:90:timeout -s KILL 80 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/sq1 -o sq1 -- tools/bin/wc_bench $W" \
 "kt:90:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt -o kt -- tools/bin/wc_bench $W"
