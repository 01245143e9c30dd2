#!/bin/bash
# Round 6: the HBM ceiling at each kernel's read:write mix (tools/bw_probe.hip, 4 GiB per launch,
# best of 10).  Mixes: 1:0 read only, 0:1 write only, 5:1 (C2 K1: 2.15 read + 0.41 staged),
# 2:1 (C5 K1), 1:1 (K6r: 0.99 + 1.07), 1:2 (the emit: 0.35 + 0.65).  Plain and nontemporal
# loads / stores (the product's K1: NT loads + NT stores; emit: NT loads, plain stores).
# Prediction: read-only ~6.3 TB/s, write-only ~5.2 (r04 mall_probe), mixes in between; the
# product kernels' counter traffic (K1 6.0, emit 4.9, K6r 6.3 TB/s at C2) within 5 % of their mix.
for r in 1 2; do
  for pq in "1 0" "0 1" "5 1" "2 1" "1 1" "1 2"; do
    for nt in "0 0" "1 0" "0 1" "1 1"; do
      timeout -k 5 60 tools/bin/bw_probe $pq 4096 $nt 10 || exit 1
    done
  done
done
