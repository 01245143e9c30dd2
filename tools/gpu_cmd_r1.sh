set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t4.log 2>&1; echo "tests rc=$?"
for d in 0 1; do echo "== dbg=$d"; WCAMD_DBG=$d timeout -k 10 60 tools/bin/wc_bench 1024 64 f64 0.999 10 2 1 || exit 1; done > gpurun_out/inv4.log 2>&1 && echo DONE
