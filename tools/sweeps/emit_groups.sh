# Shapes after the grouped reverse-order emit dispatch (compare DESIGN.md matrix).
for a in "1024 64 f64 0.999" "1024 64 f32 0.999" "128 128 f64 0.9999" "64 128 f32 0.9999" "8192 32 f64 0.999"; do
  echo "$a: $(timeout -k 5 60 tools/bin/wc_bench $a 30 3 0 0 1 | grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {.*}\|"paths_identical": [0-9]' | tr '\n' ' ')"
done
