set -o pipefail
exec tools/gpu_run.sh \
  "gputest:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "f32_128:120:tools/bin/wc_bench 64 128 f32 0.9999 20 3 0 0 1" \
  "f32_64:120:tools/bin/wc_bench 1024 64 f32 0.999 20 3 0 0 1"
