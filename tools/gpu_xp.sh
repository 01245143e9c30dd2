#!/bin/bash
# A/B of diagnostic libwavelet_amd.so variants (tools/build_variants.sh) on the inverse
A="1024 64 f64 0.999 20 3 1 0 1 1 1"
for v in default nostore nopairs neither default; do
  if [ $v = default ]; then lp=""; else lp="tools/variants/$v"; fi
  echo "$v: $(LD_LIBRARY_PATH=$lp timeout -k 5 60 tools/bin/wc_bench $A | grep -o '"inverse_stage_ms": {.*}')"
done
