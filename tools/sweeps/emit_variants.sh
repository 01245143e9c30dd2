# A/B of libwavelet_amd.so variants (tools/build_variants.sh) on the headline and C5 shapes.
for rep in 1 2 3; do
for v in default ordered; do
  if [ $v = default ]; then lp=""; else lp="tools/variants/$v"; fi
  for a in "1024 64 f64 0.999" "64 128 f32 0.9999"; do
    echo "$v $a: $(LD_LIBRARY_PATH=$lp timeout -k 5 60 tools/bin/wc_bench $a 30 3 0 0 1 | grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {.*}\|"paths_identical": [0-9]' | tr '\n' ' ')"
  done
done
done
