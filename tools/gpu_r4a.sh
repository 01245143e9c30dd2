#!/bin/bash
# Round 4, call 6: counter traffic of the cohort forward (does the ring stay
# on-die?), the full -m gpu suite, and the bench line with the new legs.
S=tools/bin/wc_bench
A="512 128 f32 0.9999 3 1 0 0"
steps=()
for v in default plain; do
  L=""; [ $v != default ] && L="LD_LIBRARY_PATH=tools/variants/$v"
  steps+=("pmc_${v}_fetch:90:$L WCB_COHORT=4 WCB_COHORT_LAG=2 timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_coh_$v -o fetch -- $S $A")
  steps+=("pmc_${v}_write:90:$L WCB_COHORT=4 WCB_COHORT_LAG=2 timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_coh_$v -o write -- $S $A")
done
steps+=("tests:700:python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread")
steps+=("bench:400:python bench.py > gpurun_out/bench_line.txt")
exec tools/gpu_run.sh "${steps[@]}"
