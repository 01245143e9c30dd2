#!/bin/bash
# One GPU call for a round's profiles: the -m gpu suite, the FETCH_SIZE and
# WRITE_SIZE passes and kernel trace of the torch-free driver (forward +
# inverse), their summary (gpurun_out/pmc_forward.json, same kernel sources),
# the default bench line carrying that traffic, and the kernel trace of
# bench.py.  CLI=1 adds the end-to-end CLI timing.  Every step has its own limit.
W="${WCB_ARGS:-1024 64 f64 0.999}"
steps=(
  "gputest:400:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread"
  "pmc_fetch:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- tools/bin/wc_bench $W 3 1 1 0"
  "pmc_write:120:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- tools/bin/wc_bench $W 3 1 1 0"
  "kt_wcb:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wcb -o wcb -- tools/bin/wc_bench $W 10 2 1 0"
  "pmc_sum:60:python tools/pmc_summary.py gpurun_out/prof_wcb/wcb_kernel_stats.csv --fetch gpurun_out/prof_fetch/fetch_counter_collection.csv --write gpurun_out/prof_write/write_counter_collection.csv --out gpurun_out/pmc_forward.json"
  "bench:400:python bench.py --pmc gpurun_out/pmc_forward.json > gpurun_out/bench_line.txt"
  "kt_bench:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline"
)
[ "${CLI:-0}" = 1 ] && steps+=("cli:600:python tools/bench_cli.py --scale 1.0 --ncomp 4 --out gpurun_out/cli_e2e.json")
exec tools/gpu_run.sh "${steps[@]}"
