set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t2.log 2>&1 && echo TESTS_OK &&
timeout -k 10 300 tools/chunk_sweep.sh > gpurun_out/c2.log 2>&1 <<'L'
0 3 0 256
0 3 64 256
0 3 64 256
L
echo SWEEP_DONE
