#!/bin/bash
# One GPU call for a round's profiles (run through gpurun; every step has its
# own limit, tools/gpu_run.sh):
#   per workload: FETCH_SIZE and WRITE_SIZE passes (separate runs) and a
#   --kernel-trace --stats run of the torch-free driver on the workload's path,
#   summarised to gpurun_out/pmc/pmc_<workload>.json (tools/pmc_summary.py);
#   then the default bench line carrying that traffic, the kernel trace of
#   bench.py itself, and (DROPIN=1) the drop-in driver, (CLI=1) the end-to-end
#   CLI, (GPUTEST=1) the -m gpu suite.
# Paths (tools/wc_bench.hip inv_mode): c4 forward only; c2 / c5 / f32_64 forward + wc_inverse
# (row index kernel + K6r), c3 wc_forward_rows + wc_inverse_rows with the fused
# RMSE (the bench's C3 round-trip leg: no row index kernel).
# usage: tools/gpu_profile.sh [workload ...]   (default: c2 c3 c5 f32_64 c4)
#   send as: gpurun -- "WC_GIT=$(git rev-parse --short HEAD) tools/gpu_profile.sh" (the box's
#   copy has no .git; the summaries record that commit)
set -o pipefail
# c4: the C3 layout with 80 units per box (10 timesteps x 8 components), forward only
# c4_hist: the same C4 batch in the opt-in global-threshold mode (WCB_HIST: stage with the
# histogram, threshold, emit; bench.py's c4.global_hist leg at its default quantile 0.7)
declare -A ARGS=([c2]="1024 64 f64 0.999" [c3]="4 c3 f64 0.999" [c5]="512 128 f32 0.9999" [f32_64]="1024 64 f32 0.999" [c4]="80 c3 f64 0.999" [c4_hist]="80 c3 f64 0.999")
declare -A MODE=([c2]=1 [c3]=3 [c5]=1 [f32_64]=1 [c4]=0 [c4_hist]=0)
declare -A DT=([c2]=f64 [c3]=f64 [c5]=f32 [f32_64]=f32 [c4]=f64 [c4_hist]=f64)
declare -A ENVS=([c4_hist]="WCB_HIST=0.7")
wls=("$@")
[ ${#wls[@]} -eq 0 ] && wls=(c2 c3 c5 f32_64 c4 c4_hist)
# summaries of workloads not profiled in this call: the committed ones (same sources only, bench.py checks)
steps=("seed:30:mkdir -p gpurun_out/pmc && (cp profiles/r06/pmc_*.json gpurun_out/pmc/ 2>/dev/null; true)")
for w in "${wls[@]}"; do
  a="${ARGS[$w]}"; m="${MODE[$w]}"; d="gpurun_out/prof_$w"; ev="${ENVS[$w]:-}"
  # counter runs: 3 timed + 1 warm-up executions of the path
  steps+=("pmcf_$w:120:$ev timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d -o fetch -- tools/bin/wc_bench $a 3 1 $m 0")
  steps+=("pmcw_$w:120:$ev timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d -o write -- tools/bin/wc_bench $a 3 1 $m 0")
  steps+=("kt_$w:200:$ev rocprofv3 --kernel-trace --stats --output-format csv -d $d -o kt -- tools/bin/wc_bench $a 10 2 $m 0")
  steps+=("sum_$w:60:mkdir -p gpurun_out/pmc && python tools/pmc_summary.py $d/kt_kernel_stats.csv --fetch $d/fetch_counter_collection.csv --write $d/write_counter_collection.csv --steps 4 --workload $w --dtype ${DT[$w]} --note 'tools/gpu_profile.sh: wc_bench $a inv_mode $m, FETCH_SIZE x2 + WRITE_SIZE per dispatch' --out gpurun_out/pmc/pmc_$w.json")
done
steps+=("bench:500:python bench.py --pmc gpurun_out/pmc > gpurun_out/bench_line.txt")
steps+=("kt_bench:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --pmc gpurun_out/pmc")
[ "${DROPIN:-0}" = 1 ] && steps+=("dropin:600:tools/bin/dropin_bench /tmp/wcamd_dropin_\$\$ 4 0.999 > gpurun_out/dropin.json")
[ "${CLI:-0}" = 1 ] && steps+=("cli:600:python tools/bench_cli.py --scale 1.0 --ncomp 4 --out gpurun_out/cli_e2e.json")
[ "${GPUTEST:-0}" = 1 ] && steps+=("gputest:500:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
exec tools/gpu_run.sh "${steps[@]}"
