#!/bin/bash
# One GPU call for a round's profiles: the -m gpu suite, the default bench line,
# the headline profiles (kernel trace of bench.py, torch-free driver trace,
# FETCH_SIZE and WRITE_SIZE passes of forward + inverse), and the end-to-end CLI
# timing.  Every step has its own time limit.
W="${WCB_ARGS:-1024 64 f64 0.999}"
exec tools/gpu_run.sh \
  "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "bench:400:python bench.py" \
  "kt_bench:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline" \
  "kt_wcb:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wcb -o wcb -- tools/bin/wc_bench $W 10 2 1 0" \
  "pmc_fetch:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- tools/bin/wc_bench $W 3 1 1 0" \
  "pmc_write:120:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- tools/bin/wc_bench $W 3 1 1 0" \
  "cli:600:python tools/bench_cli.py --scale 1.0 --ncomp 4 --out gpurun_out/cli_e2e.json"
