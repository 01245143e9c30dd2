# The row index's (K5) run loads nontemporal (WC_RIX_RUNS_NT): the -d form of the inverse
for r in 1 2 3 4; do
  for v in base runsnt; do
    L=tools/variants/$v
    echo "$v c2m1"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 30 3 1 0 || exit 1
    echo "$v c5m1"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 512 128 f32 0.9999 10 2 1 0 || exit 1
  done
done
