#!/bin/bash
# Round 4: persistent, software-pipelined S32 K1 (WC_OPT_K1_PERSIST 1: the next
# tile's cells load during the current tile's phase 2) vs one workgroup per
# tile (WCB_K1PF=0); C2 fp64, fp32 64^3, C5; forward only, alternated 3 times;
# a full-batch check against the conservative path; the parity suite.
S=tools/bin/wc_bench
steps=()
for r in 1 2 3; do
  for k in 1 0; do
    steps+=("pf${k}_c2_$r:90:WCB_K1PF=$k $S 1024 64 f64 0.999 10 2 0 0")
    steps+=("pf${k}_f32_$r:90:WCB_K1PF=$k $S 1024 64 f32 0.999 10 2 0 0")
    steps+=("pf${k}_c5_$r:90:WCB_K1PF=$k $S 512 128 f32 0.9999 10 2 0 0")
  done
done
steps+=("check_c2:120:$S 1024 64 f64 0.999 3 1 1 1")
steps+=("check_c5:120:$S 512 128 f32 0.9999 3 1 0 1")
steps+=("tests:600:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread")
exec tools/gpu_run.sh "${steps[@]}"
