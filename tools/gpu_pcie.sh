#!/bin/bash
# PCIe / host-copy probe (tools/pcie_probe.cpp) beside the bench.py host leg on the same box.
exec tools/gpu_run.sh \
  "pcie_probe:150:tools/bin/pcie_probe" \
  "host_leg:240:python bench.py --legs host --no-cpu-baseline --steps 3 --warmup 1 --leg-steps 5"
