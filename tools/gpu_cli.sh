#!/bin/bash
exec tools/gpu_run.sh "cli:600:python tools/bench_cli.py --scale 1.0 --ncomp 4 --out gpurun_out/cli_e2e.json"
