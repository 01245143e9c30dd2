#!/bin/bash
# The driver's N = 8 code path rehearsed on one GPU: 8 ranks (gloo; the default
# launch-order look-backs, 8 processes' kernels sharing the device), every default
# leg, C4/C5 sharded over 8 ranks, one merged line.
exec tools/gpu_run.sh \
  "rehearse8:900:python bench.py --gpus 8 --rehearse --no-cpu-baseline --steps 3 --warmup 1 --leg-steps 2 > gpurun_out/rehearse_8ranks.txt"
