#!/bin/bash
# FETCH_SIZE of the inverse kernels: XCD-grouped K6r order (default) vs unit order.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_rx -o def -- tools/bin/wc_bench 1024 64 f64 0.999 3 1 1 0 1 1 1 > gpurun_out/pmc_rx_def.log 2>&1 &&
LD_LIBRARY_PATH=tools/variants/rixnat timeout -k 10 -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_rx -o nat -- tools/bin/wc_bench 1024 64 f64 0.999 3 1 1 0 1 1 1 > gpurun_out/pmc_rx_nat.log 2>&1 &&
LD_LIBRARY_PATH=tools/variants/rixnat timeout -k 10 -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_rx -o nat32 -- tools/bin/wc_bench 8192 32 f64 0.999 3 1 1 0 1 1 1 > gpurun_out/pmc_rx_nat32.log 2>&1 &&
timeout -k 10 -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_rx -o def32 -- tools/bin/wc_bench 8192 32 f64 0.999 3 1 1 0 1 1 1 > gpurun_out/pmc_rx_def32.log 2>&1
