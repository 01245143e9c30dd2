#!/bin/bash
# Quick forward check: C2 / C5 wc_bench (with the conservative-path comparison) + forward parity tests.
exec tools/gpu_run.sh \
 "wcb_c2:120:tools/bin/wc_bench 1024 64 f64 0.999 20 3 0 1" \
 "wcb_c5:120:tools/bin/wc_bench 64 128 f32 0.9999 20 3 0 1" \
 "wcb_c2b:120:tools/bin/wc_bench 1024 64 f64 0.999 20 3 0 0" \
 "fwdtest:300:python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k 'forward_payload or special or unaligned or empty'"
