#!/bin/bash
# Chunked-forward diagnostic (wc_bench WCB_CHUNK: the batch as calls of k units
# sharing one k-unit staging buffer: is the staging round trip cheaper when it
# stays in the Infinity Cache?), then tools/gpu_profile3.sh with the -m gpu suite.
S=tools/bin/wc_bench
steps=()
for k in 0 4 8 16; do
  steps+=("c5_chunk$k:90:WCB_CHUNK=$k $S 512 128 f32 0.9999 10 2 0 0")
done
for k in 0 16 32 64; do
  steps+=("c2_chunk$k:90:WCB_CHUNK=$k $S 1024 64 f64 0.999 10 2 0 0")
done
tools/gpu_run.sh "${steps[@]}" && TESTS=1 exec tools/gpu_profile3.sh
