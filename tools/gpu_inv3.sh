#!/bin/bash
# Row index over the device-built item list: parity, timings, kernel trace, K6r diagnostic variants.
S="tools/bin/wc_bench"
A="1024 64 f64 0.999 20 3 1 0 1 1 1"
B="64 128 f32 0.9999 20 3 1 0 1 1 1"
steps=()
for v in nostore nopairs noscans nophasec; do
  steps+=("v_${v}_c2:60:LD_LIBRARY_PATH=tools/variants/$v $S $A")
  steps+=("v_${v}_c5:60:LD_LIBRARY_PATH=tools/variants/$v $S $B")
done
exec tools/gpu_run.sh \
 "invtest:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread" \
 "c2_check:120:$S 1024 64 f64 0.999 5 2 1 1 1 1 1" \
 "c2:60:$S $A" "c5:60:$S $B" \
 "c2_tk:60:$S 1024 64 f64 0.999 20 3 1 0 0 1 1" \
 "s16:60:$S 32768 16 f64 0.999 20 3 1 0 1 1 1" \
 "s32:60:$S 8192 32 f64 0.999 20 3 1 0 1 1 1" \
 "kt:120:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_inv -o inv -- $S 1024 64 f64 0.999 10 2 1 0" \
 "${steps[@]}"
