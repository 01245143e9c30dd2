"""wc_inverse_host one run vs pipelined runs (WC_OPT_HOST_CHUNK) on C2
(1024 x 64^3 fp64, keep 0.999f): ms per call, PCIe-inclusive."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import wcamd  # noqa: E402
from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK  # noqa: E402

wc = wcamd
n, D = 1024, 64
rng = np.random.default_rng(1)
units, n, extent = wc.capi.make_units([(D, D, D)] * n)
cells = np.empty(extent, np.float64)
base = rng.standard_normal(D ** 3)
for i in range(n):  # cheap distinct boxes: a shared field, scaled and shifted per box
    cells[i * D ** 3:(i + 1) * D ** 3] = base * (1 + 0.01 * i) + 0.001 * i
ctx = wc.capi.Context(0)
keep = float(np.float32(0.999))
payload, offs, kept = ctx.forward_host(cells, units, n, keep)
ref = None
for chunk in [0, 1 << 25, 1 << 24, 0, 1 << 25, 1 << 24]:
    ctx.set_option(WC_OPT_HOST_CHUNK, chunk)
    out = ctx.inverse_host(payload, offs[:n], units, n, extent)
    if ref is None:
        ref = out.copy()
    assert np.array_equal(out, ref), chunk
    t0 = time.perf_counter()
    for _ in range(5):
        ctx.inverse_host(payload, offs[:n], units, n, extent)
    print(f"chunk {chunk}: inverse_host {(time.perf_counter() - t0) / 5 * 1e3:.1f} ms", flush=True)
