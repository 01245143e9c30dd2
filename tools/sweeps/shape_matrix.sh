# DESIGN.md shape/dtype/keep matrix: forward + inverse per row (wc_bench inverse=1), then check=1 parity.
for a in "1024 64 f64 0.999" "1024 64 f32 0.999" "128 128 f64 0.9999" "64 128 f32 0.9999" "8192 32 f64 0.999" "1024 64 f64 0.99" "1024 64 f64 0.9999"; do
  timeout -k 5 60 tools/bin/wc_bench $a 30 3 1 0 0 || exit $?
  echo "check $a: $(timeout -k 5 60 tools/bin/wc_bench $a 3 1 0 0 1 | grep -o '"paths_identical": [0-9]')"
done
