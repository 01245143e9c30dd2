#!/bin/bash
# -m gpu suite, then the forward/inverse of C2 and C5 through wc_bench (check=1
# against the conservative paths), then the default bench line.
S=tools/bin/wc_bench
exec tools/gpu_run.sh \
  "tests:700:python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread" \
  "c2:60:$S 1024 64 f64 0.999 10 2 1 1" \
  "c2b:60:$S 1024 64 f64 0.999 10 2 1 0" \
  "c5:90:$S 512 128 f32 0.9999 10 2 1 0" \
  "bench:400:python bench.py --pmc none > gpurun_out/bench_line.txt"
