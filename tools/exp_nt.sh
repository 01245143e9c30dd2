# Nontemporal stores / loads of the streaming data (profiles/r05/experiments/gpu_nt.txt): K1 staged
# coefficients (WC_K1_NT_STAGE), K6r x-quad output (WC_RIX_NT), emit staged-coefficient loads
# (WC_EMIT_NTLOAD); krP used a K6r pair-load toggle since removed (measured slower)
for r in 1 2 3 4; do
  for v in base kr krE krP; do
    L=tools/variants/$v
    echo "$v c2"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 40 5 1 0 || exit 1
    echo "$v c2r"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f64 0.999 40 5 3 0 || exit 1
    echo "$v c3"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 4 c3 f64 0.999 40 5 3 0 || exit 1
    echo "$v c5"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 512 128 f32 0.9999 15 3 1 0 || exit 1
    echo "$v f32_64"; LD_LIBRARY_PATH=$L timeout -k 5 60 tools/bin/wc_bench 1024 64 f32 0.999 40 5 1 0 || exit 1
  done
done
