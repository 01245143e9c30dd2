"""wc_forward_host / wc_inverse_host with and without the destination prefault
(WC_OPT_HOST_THREADS, WC_OPT_HOST_THP) on C2 (1024 x 64^3 fp64 cells in
pinned host memory, keep 0.999f; payloads and boxes into fresh pageable
arrays, as capi.Context allocates them): ms per call, PCIe-inclusive, and
every setting's bytes equal to the first's.

Predicted (tools/pcie_probe.cpp, profiles/r04/experiments/gpu_pcie.txt): the
forward falls from ~76 ms to the 2.15 GB upload, ~38-42 ms; the inverse from
~121 ms to the 1.07 GB download, ~20-25 ms."""
import json
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench_workloads as bw  # noqa: E402
import wcamd  # noqa: E402
from wavelet_compression_amd.capi import WC_OPT_HOST_THP, WC_OPT_HOST_THREADS  # noqa: E402

wc = wcamd
dev = torch.device("cuda", 0)
units = bw.WORKLOADS["c2"]["units"]()
cells_dev, offs_cells, extent = bw.synth_cells(torch, dev, units, "f64")
tab, n, _ = bw.units_array(wc.capi, units, offs_cells)
pinned = torch.empty(cells_dev.numel(), dtype=cells_dev.dtype, pin_memory=True)
pinned.copy_(cells_dev)
torch.cuda.synchronize()
del cells_dev
torch.cuda.empty_cache()
arr = pinned.numpy()
keep = float(np.float32(0.999))
ctx = wc.capi.Context(0)
print(json.dumps({"default_threads": None}), flush=True)
ref = None
for rep in range(2):
    for threads, thp in [(0, 0), (-1, 1), (-1, 0), (4, 1), (0, 1)]:
        ctx.set_option(WC_OPT_HOST_THREADS, threads)
        ctx.set_option(WC_OPT_HOST_THP, thp)
        eff = ctx.get_option(WC_OPT_HOST_THREADS)
        payload, offs, kept = ctx.forward_host(arr, tab, n, keep)  # warm-up (host staging buffers)
        fw = []
        for _ in range(4):
            t0 = time.perf_counter()
            payload, offs, kept = ctx.forward_host(arr, tab, n, keep)
            fw.append((time.perf_counter() - t0) * 1e3)
        out = ctx.inverse_host(payload, offs[:n], tab, n, arr.size)
        inv = []
        for _ in range(4):
            t0 = time.perf_counter()
            out = ctx.inverse_host(payload, offs[:n], tab, n, arr.size)
            inv.append((time.perf_counter() - t0) * 1e3)
        end = int(offs[n])
        if ref is None:
            ref = (payload[:end].copy(), offs.copy(), kept.copy(), out.copy())
        same = (np.array_equal(ref[0], payload[:end]) and np.array_equal(ref[1], offs)
                and np.array_equal(ref[2], kept) and np.array_equal(ref[3], out))
        print(json.dumps({"rep": rep, "threads": eff, "thp": thp, "forward_ms": [round(x, 2) for x in fw],
                          "inverse_ms": [round(x, 2) for x in inv], "payload_bytes": end, "same_bytes": bool(same)}),
              flush=True)
        assert same
