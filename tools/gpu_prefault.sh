#!/bin/bash
# Host-buffer calls (wc_forward_host / wc_inverse_host): host parity tests,
# the library's host-side timeline (tools/host_trace.py), the A/B over the
# destination prefault settings, the bench.py host leg.
exec tools/gpu_run.sh \
  "host_tests:300:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'host or prefault'" \
  "host_trace:200:python -u tools/host_trace.py" \
  "prefault_ab:300:python -u tools/host_prefault_ab.py" \
  "host_leg:240:python bench.py --legs host --no-cpu-baseline --steps 3 --warmup 1 --leg-steps 5"
