#!/bin/bash
# A/B of diagnostic libwavelet_amd.so variants (tools/build_variants.sh) on the forward.
for A in "1024 64 f64 0.999 20 3 0 0 1 1 1" "64 128 f32 0.9999 20 3 0 0 1 1 1"; do
for v in default $VARIANTS; do
  if [ $v = default ]; then lp=""; else lp="tools/variants/$v"; fi
  echo "$A $v: $(LD_LIBRARY_PATH=$lp timeout -k 5 60 tools/bin/wc_bench $A | grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {.*}' | tr '\n' ' ')"
done
done
