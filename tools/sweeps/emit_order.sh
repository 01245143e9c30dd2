# Emit dispatch order sweep (WC_EMIT_GROUP / WC_EMIT_REV), 1024 x 64^3 fp64 and 64 x 128^3 fp32.
for rep in 1 2; do
for cfg in "1024 0" "256 1" "256 0" "512 1" "384 1"; do
  set -- $cfg
  echo "64^3 group=$1 rev=$2: $(WC_EMIT_GROUP=$1 WC_EMIT_REV=$2 timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 30 3 0 0 1 | grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {.*}\|"paths_identical": [0-9]' | tr '\n' ' ')"
done
done
for cfg in "64 0" "32 1" "16 1" "8 1"; do
  set -- $cfg
  echo "128^3 f32 group=$1 rev=$2: $(WC_EMIT_GROUP=$1 WC_EMIT_REV=$2 timeout -k 5 60 tools/bin/wc_bench 64 128 f32 0.9999 30 3 0 0 1 | grep -o '"ms_per_step": [0-9.]*\|"stage_ms": {.*}\|"paths_identical": [0-9]' | tr '\n' ' ')"
done
