"""Diagnostic (round 6): NaN bits of the GPU inverse where the reference's
x86 arithmetic makes an invalid-operation NaN (inf - inf): boxes with one
-inf or +inf cell, everything kept, odd and even dims, through wc_inverse and
wc_inverse_rows; prints the NaN bit patterns of the GPU and the oracle."""
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "oracle"))
import wcamd as wc  # noqa: E402
import oracle as O  # noqa: E402

ctx = wc.capi.Context(0)
for dims in ((4, 2, 2), (3, 2, 2), (4, 4, 8), (33, 8, 33), (8, 8, 8)):
    W, H, D = dims
    for v in (-np.inf, np.inf):
        b = np.random.default_rng(1).standard_normal((D, H, W)).astype(np.float32) * 100
        b[D // 2, H // 2, W // 2] = v
        units, n, ext = wc.capi.make_units([dims])
        pay, po, kept = ctx.forward_host(b.ravel(), units, n, 0.5)
        got = ctx.inverse_host(pay, po, units, n, ext)
        want = O.decompress_payload(wc.capi.unit_payload(pay, po, kept, 0)).ravel()
        gb = got.view(np.uint32)[np.isnan(got)]
        wb = want.view(np.uint32)[np.isnan(want)]
        print(dims, v, "kept", int(kept[0]), "gpu nan bits", sorted(set(hex(x) for x in gb)),
              "oracle nan bits", sorted(set(hex(x) for x in wb)), "equal", got.tobytes() == want.tobytes())
