#!/bin/bash
# Multi-rank rehearsal on one GPU (2 ranks, gloo, both on device 0) + end-to-end CLI timing.
exec tools/gpu_run.sh \
 "rehearse2:400:python bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --leg-steps 2 --no-cpu-baseline" \
 "cli:600:python tools/bench_cli.py --scale 1.0 --ncomp 4 --out gpurun_out/cli_e2e.json"
