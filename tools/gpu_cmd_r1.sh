set -o pipefail
exec tools/gpu_run.sh \
  "nt64:120:tools/bin/wc_bench 1024 64 f64 0.999 20 3 0 0 1" \
  "nt32:120:tools/bin/wc_bench 64 128 f32 0.9999 20 3 0 0 1"
