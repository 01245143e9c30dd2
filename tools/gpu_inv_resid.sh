#!/bin/bash
# Round 4: is the row-indexed inverse HBM-bound?  K6r time per unit when the
# batch's payload (just read by the row index) fits the 256 MiB Infinity Cache
# vs when it does not; then the SQ cycle split of K5/K6r at the C5 shape.
S=tools/bin/wc_bench
steps=()
for nb in 1024 512 256 128; do steps+=("c2inv_$nb:90:$S $nb 64 f64 0.999 10 2 1 0"); done
for nb in 512 128 32 16; do steps+=("c5inv_$nb:90:$S $nb 128 f32 0.9999 10 2 1 0"); done
P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
steps+=("sq_c5inv:90:timeout -s KILL 80 rocprofv3 --pmc $P --output-format csv -d gpurun_out/sq4 -o c5 -- $S 512 128 f32 0.9999 3 1 1 0")
exec tools/gpu_run.sh "${steps[@]}"
