# K6r second-round prefetch A/B (variants under tools/variants/)
for v in base r12s4 r8s8 r12s0; do
  L=tools/variants/$v
  for r in 1 2; do
    echo "$v c2 mode1"; LD_LIBRARY_PATH=$L tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 0
    echo "$v c3 mode6"; LD_LIBRARY_PATH=$L tools/bin/wc_bench 4 c3 f64 0.999 20 3 6 0
    echo "$v c3 mode3"; LD_LIBRARY_PATH=$L tools/bin/wc_bench 4 c3 f64 0.999 20 3 3 0
    echo "$v c5 mode1"; LD_LIBRARY_PATH=$L tools/bin/wc_bench 512 128 f32 0.9999 10 2 1 0
  done
done
