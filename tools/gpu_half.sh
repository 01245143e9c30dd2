#!/bin/bash
# Timing probe: staging only the first half (64 B) of each 32-coefficient segment (wrong bytes, timing only).
S="tools/bin/wc_bench"
steps=()
for cfg in "1024 64 f64 0.999" "64 128 f32 0.9999" "1024 64 f64 0.9999"; do
  set -- $cfg; n="$1_$2_$4"
  steps+=("def_$n:60:$S $cfg 20 3 0 0 1 1 1")
  steps+=("half_$n:60:LD_LIBRARY_PATH=tools/variants/half $S $cfg 20 3 0 0 1 1 1")
  steps+=("wr_$n:60:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pw_$n -o w -- $S $cfg 3 1 0 0 1 1 1")
  steps+=("wrh_$n:60:LD_LIBRARY_PATH=tools/variants/half rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pwh_$n -o w -- $S $cfg 3 1 0 0 1 1 1")
  steps+=("fe_$n:60:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pf_$n -o f -- $S $cfg 3 1 0 0 1 1 1")
  steps+=("feh_$n:60:LD_LIBRARY_PATH=tools/variants/half rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pfh_$n -o f -- $S $cfg 3 1 0 0 1 1 1")
done
exec tools/gpu_run.sh "${steps[@]}"
