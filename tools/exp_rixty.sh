# K6r tile rows by runtime option (round 5): WC_OPT_RIX_LDS 4608 gives TX 16, TY 1 at D = 64
# (64-coefficient ranges: every range one 64-pair round; tiles of half the cells) vs the default
# 9216 (TX 16, TY 2).  At D = 128 (C5) the smaller budget narrows x to 8 blocks instead.
for r in 1 2 3; do
  for cfg in "9216 4" "4608 4"; do
    set -- $cfg
    echo "lds=$1 tx=$2 c3m3"; timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 30 3 3 0 1 1 1 $1 $2 || exit 1
    echo "lds=$1 tx=$2 c2m3"; timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 30 3 3 0 1 1 1 $1 $2 || exit 1
    echo "lds=$1 tx=$2 c2m1"; timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 30 3 1 0 1 1 1 $1 $2 || exit 1
    echo "lds=$1 tx=$2 c5m1"; timeout -k 5 60 tools/bin/wc_bench 512 128 f32 0.9999 10 2 1 0 1 1 1 $1 $2 || exit 1
  done
done
