"""Host-side timeline of wc_forward_host / wc_inverse_host on C2 (WCAMD_HOST_TRACE=1
prints the library's marks to stderr); the Python-level call and the free of
the previous result are timed around them."""
import os
import sys
import time

import numpy as np

os.environ["WCAMD_HOST_TRACE"] = "1"
sys.path.insert(0, ".")
import torch  # noqa: E402

import bench_workloads as bw  # noqa: E402
import wcamd  # noqa: E402

wc = wcamd
dev = torch.device("cuda", 0)
units = bw.WORKLOADS["c2"]["units"]()
cells_dev, offs_cells, extent = bw.synth_cells(torch, dev, units, "f64")
tab, n, _ = bw.units_array(wc.capi, units, offs_cells)
pinned = torch.empty(cells_dev.numel(), dtype=cells_dev.dtype, pin_memory=True)
pinned.copy_(cells_dev)
torch.cuda.synchronize()
arr = pinned.numpy()
if os.environ.get("HOST_TRACE_PAGEABLE"):  # cells in ordinary (pageable) host memory, as a C++ caller's vector
    arr = arr.copy()
    print("pageable cells", file=sys.stderr, flush=True)
keep = float(np.float32(0.999))
ctx = wc.capi.Context(0)
for it in range(3):
    t0 = time.perf_counter()
    payload, offs, kept = ctx.forward_host(arr, tab, n, keep)
    t1 = time.perf_counter()
    print(f"forward_host call {(t1 - t0) * 1e3:.2f} ms", file=sys.stderr, flush=True)
    out = ctx.inverse_host(payload, offs[:n], tab, n, arr.size)
    t2 = time.perf_counter()
    print(f"inverse_host call {(t2 - t1) * 1e3:.2f} ms", file=sys.stderr, flush=True)
    del out
    t3 = time.perf_counter()
    del payload
    t4 = time.perf_counter()
    print(f"free out {(t3 - t2) * 1e3:.2f} ms, free payload {(t4 - t3) * 1e3:.2f} ms", file=sys.stderr, flush=True)
    t5 = time.perf_counter()
    e = np.empty(int(wc.capi.payload_bound(tab, n)), np.uint8)
    t6 = time.perf_counter()
    print(f"np.empty(bound) {(t6 - t5) * 1e3:.2f} ms", file=sys.stderr, flush=True)
    del e
