#!/bin/bash
# GPU check of the current tree: the -m gpu suite, then the default bench line.
exec tools/gpu_run.sh \
 "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "bench:400:python bench.py" \
 "wcb_c2:120:tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 1" \
 "wcb_c5:120:tools/bin/wc_bench 64 128 f32 0.9999 20 3 1 1"
