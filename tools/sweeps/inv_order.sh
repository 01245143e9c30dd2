# Inverse order sweep: decode interleave groups (WC_DEC_GROUP units) x inverse reverse order (WC_INV_REV).
for rep in 1 2; do
for cfg in "1024 0" "1024 1" "128 1" "256 1" "64 1" "256 0"; do
  set -- $cfg
  echo "64^3 dgroup=$1 rev=$2: $(WC_DEC_GROUP=$1 WC_INV_REV=$2 timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 30 3 1 0 0 | grep -o '"inverse[a-z_]*": [{0-9.][^}]*' | tr '\n' ' ')"
done
done
