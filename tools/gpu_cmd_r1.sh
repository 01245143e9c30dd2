set -o pipefail
exec tools/gpu_run.sh \
  "kt_wcb:200:rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wcb -o wcb -- tools/bin/wc_bench 1024 64 f64 0.999 10 2 1" \
  "pmc_fetch:200:rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o fetch -- tools/bin/wc_bench 1024 64 f64 0.999 3 1 1" \
  "pmc_write:200:rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof_write -o write -- tools/bin/wc_bench 1024 64 f64 0.999 3 1 1" \
  "wcb_f32:120:tools/bin/wc_bench 64 128 f32 0.9999 10 2 1 0 1"
