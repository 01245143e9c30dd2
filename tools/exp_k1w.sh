# K1 write cost diagnostic (round 5): staged coefficient stores suppressed (nostore, results
# invalid), flag stores suppressed (noflag, invalid), staging written tile-major (tmaj: each K1
# tile's rows in one contiguous 32 KB region; the emit then reads garbage; C2 shape only), dense staging
for r in 1 2; do
  for v in base nostore tmaj; do
    echo "$v"; LD_LIBRARY_PATH=tools/variants/$v timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 20 3 0 0 || exit 1
  done
done
