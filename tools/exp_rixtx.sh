# K6r tile shape by runtime options (round 5): WC_OPT_RIX_LDS / WC_OPT_RIX_TX.  TX 32 blocks with
# TY 1 row per range (64-coefficient ranges: one 64-pair round always) vs the default TX 16, TY 2.
for r in 1 2; do
  for cfg in "9216 4" "9216 5" "12288 5" "18432 5"; do
    set -- $cfg
    echo "lds=$1 tx=$2 c3m3"; tools/bin/wc_bench 4 c3 f64 0.999 20 3 3 0 1 1 1 $1 $2
    echo "lds=$1 tx=$2 c2m1"; tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 0 1 1 1 $1 $2
    echo "lds=$1 tx=$2 c5m1"; tools/bin/wc_bench 512 128 f32 0.9999 10 2 1 0 1 1 1 $1 $2
  done
done
