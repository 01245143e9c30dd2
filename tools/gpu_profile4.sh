#!/bin/bash
# Round-4 counter summaries, one per workload (bench.py --pmc reads pmc_*.json):
#   c2      1024 x 64^3 fp64, keep 0.999f, forward + inverse (wc_inverse)
#   c3      the 4-level AMR layout x 4 components, fp64, forward + fused inverse/RMSE (wc_inverse_rmse)
#   c5      512 x 128^3 fp32, keep 0.9999f, forward + inverse
#   f32_64  1024 x 64^3 fp32 (the drop-in compress() input type), keep 0.999f, forward
# per workload: FETCH_SIZE pass, WRITE_SIZE pass (separate runs: FETCH uses 3 TCC slots),
# kernel trace + stats; tools/pmc_summary.py --steps 4 (warmup 1 + 3 steps of each direction).
# Then the GPU suite and smoke (TESTS=1), the default bench line with these summaries,
# the kernel trace of bench.py, and a 2-rank rehearsal of bench.py --gpus 2 on the one GPU.
S=tools/bin/wc_bench
declare -A ARGS=([c2]="1024 64 f64 0.999" [c3]="4 c3 f64 0.999" [c5]="512 128 f32 0.9999" [f32_64]="1024 64 f32 0.999")
declare -A INV=([c2]=1 [c3]=2 [c5]=1 [f32_64]=0)
declare -A DT=([c2]=f64 [c3]=f64 [c5]=f32 [f32_64]=f32)
steps=()
[ "${TESTS:-0}" = 1 ] && steps+=("tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
                                 "smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'")
for w in ${WORKLOADS:-c2 c3 c5 f32_64}; do
  a="${ARGS[$w]}"; i="${INV[$w]}"; o="gpurun_out/pmc_$w"
  steps+=("${w}_fetch:120:timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $o -o fetch -- $S $a 3 1 $i 0")
  steps+=("${w}_write:120:timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $o -o write -- $S $a 3 1 $i 0")
  steps+=("${w}_kt:150:rocprofv3 --kernel-trace --stats --output-format csv -d $o -o kt -- $S $a 10 2 $i 0")
  steps+=("${w}_sum:60:python tools/pmc_summary.py $o/kt_kernel_stats.csv --fetch $o/fetch_counter_collection.csv --write $o/write_counter_collection.csv --steps 4 --workload $w --dtype ${DT[$w]} --note 'tools/gpu_profile4.sh: wc_bench $a, FETCH_SIZE x2 + WRITE_SIZE per dispatch' --out gpurun_out/pmc_$w.json")
done
[ "${BENCH:-1}" = 1 ] && steps+=("bench:400:python bench.py --pmc gpurun_out > gpurun_out/bench_line.txt")
[ "${KTB:-1}" = 1 ] && steps+=("kt_bench:300:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline")
[ "${REH:-1}" = 1 ] && steps+=("rehearse2:400:python bench.py --gpus 2 --rehearse --steps 5 --warmup 2 --leg-steps 2 --no-cpu-baseline --legs f32_64,c5,c4 > gpurun_out/rehearse_2ranks.txt")
exec tools/gpu_run.sh "${steps[@]}"
