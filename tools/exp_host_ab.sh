#!/bin/bash
# Round 6 host-side A/B (profiles/r06/experiments/gpu_host_ab.txt):
#  * the drop-in write-behind loop: this round's queue (per-file flush, never-destroyed, atexit drain)
#    vs round 5's (tools/variants/wbold: commit 561f7ae's write_behind.cpp, flush_writes(path) = full);
#  * the CLI -c on the C3-like plotfile as one chunk (default at one device) vs four chunks
#    (WCAMD_CHUNK_CELLS=48000000): the xz stage of chunk i beside the read + GPU pass of chunk i+1.
for r in 1 2; do
  for v in base wbold; do
    L=wavelet-compression_amd/lib; [ $v = wbold ] && L=tools/variants/wbold
    echo "$v dropin"; LD_LIBRARY_PATH=$L timeout -k 5 300 tools/bin/dropin_bench /tmp/wcamd_dropin_ab_$$ 4 0.999 || exit 1
  done
  for c in 0 48000000; do
    echo "cli chunk $c"
    if [ $c = 0 ]; then timeout -k 5 300 python tools/bench_cli.py --scale 1.0 --ncomp 4 --fast-presets 0 --out /tmp/cli_ab.json || exit 1
    else WCAMD_CHUNK_CELLS=$c timeout -k 5 300 python tools/bench_cli.py --scale 1.0 --ncomp 4 --fast-presets 0 --out /tmp/cli_ab.json || exit 1; fi
  done
done
