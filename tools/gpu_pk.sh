#!/bin/bash
# Packed-row staging probe (round 3): the packed K1/emit of c6ecaf2 as built then
# (pk0), with every packed row padded to whole 128-B lines (pkfull), and the
# same without the per-row 16-B mask writes (pknomask: timing only, payloads
# wrong), against the default flagged-segment staging; C5 shape, 2 reps.
S=tools/bin/wc_bench
A="512 128 f32 0.9999 10 2 0 0 1"
steps=("chk_pkfull:90:LD_LIBRARY_PATH=tools/variants/pkfull $S 64 128 f32 0.9999 3 1 1 1 1 2")
for rep in 1 2; do
  steps+=("ab_default_c5_$rep:90:$S $A 1")
  for v in pk0 pkfull pknomask; do steps+=("ab_${v}_c5_$rep:90:LD_LIBRARY_PATH=tools/variants/$v $S $A 2"); done
done
for v in pk0 pkfull; do
  steps+=("wr_$v:120:LD_LIBRARY_PATH=tools/variants/$v timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pk_$v -o write -- $S 512 128 f32 0.9999 3 1 0 0 1 2")
done
exec tools/gpu_run.sh "${steps[@]}"
