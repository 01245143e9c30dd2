#!/bin/bash
# Destination prefault of the _host calls (WC_OPT_HOST_THREADS / _THP): host
# parity tests, the A/B over settings (tools/host_prefault_ab.py), bench host leg.
exec tools/gpu_run.sh \
  "host_tests:300:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k 'host or prefault'" \
  "prefault_ab:300:python -u tools/host_prefault_ab.py" \
  "host_leg:240:python bench.py --legs host --no-cpu-baseline --steps 3 --warmup 1 --leg-steps 5"
