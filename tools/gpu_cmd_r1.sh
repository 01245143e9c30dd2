set -o pipefail
for c in none 24 21; do echo "== cap=$c"; if [ $c = none ]; then timeout -k 10 60 tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 || exit 1; else WCAMD_DEC_CAP=$c timeout -k 10 60 tools/bin/wc_bench 1024 64 f64 0.999 20 3 1 || exit 1; fi; done > gpurun_out/dec.log 2>&1 && echo DONE
