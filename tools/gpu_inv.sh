#!/bin/bash
# inverse redesign check: parity tests of the inverse, then wc_bench A/B
exec tools/gpu_run.sh \
 "invtest:300:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k 'inverse or rle_decode or sparse_decode or golden or format'" \
 "alltest:400:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "c2_rows:120:tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 1 1 1 1" \
 "c2_dense:120:tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 0 1 1 0" \
 "c5_rows:120:tools/bin/wc_bench 64 128 f32 0.9999 20 3 1 1 1 1 1" \
 "c5_dense:120:tools/bin/wc_bench 64 128 f32 0.9999 20 3 1 0 1 1 0" \
 "s32:120:tools/bin/wc_bench 8192 32 f64 0.999 20 3 1 1 1 1 1" \
 "s16:120:tools/bin/wc_bench 32768 16 f64 0.999 20 3 1 1 1 1 1"
