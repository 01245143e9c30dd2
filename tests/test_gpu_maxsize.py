"""The largest units the format allows, on one GPU.  ncoeff and every run are
int32 in the payload (src/compressor.cpp:55-80), so a unit holds at most
2^31 - 1 cells; the C-ABI rejects more (validate_units).  Two units near the
top, each one wc_forward + one wc_inverse_rmse:
  * 2046 x 1024 x 1024 fp32 = 2 145 386 496 cells (2^31 - 2 097 152): flat
    indices and pair counts near the int32 limit, 17 GB of payload slots, the
    row-indexed inverse (D % 8 == 0);
  * 1024 x 1024 x 1026 fp64 = 1 075 838 976 cells (> 2^30: past the 32-bit
    byte offsets of the specialised transform), hz odd (dense staging), the
    dense-decode inverse (D % 8 != 0).
The expected bytes come from tests/tiled_expect.py (each box is tiled from a
small seeded box; the oracle compresses the small box; the model is pinned
against the oracle on the CPU by tests/test_tiled_model.py): every pair of
the unit, its header, kept count and slot offsets, every reconstructed cell,
and the RMSE within 1e-9 (same terms, another summation order).
"""
import numpy as np
import pytest

from tiled_expect import TiledExpect

pytestmark = pytest.mark.gpu

KEEP = float(np.float32(0.999))

CASES = {
    "fp32_2046x1024x1024": dict(small=(62, 64, 64), big=(2046, 1024, 1024), dtype=np.float32, seed=41),
    "fp64_1024x1024x1026": dict(small=(64, 64, 54), big=(1024, 1024, 1026), dtype=np.float64, seed=43),
}


@pytest.mark.parametrize("name,path", [(n, "payload") for n in CASES] + [("fp32_2046x1024x1024", "rows")])
def test_max_size_unit_matches_tiled_oracle(wc, ctx, oracle, name, path):
    """path "payload": wc_forward + wc_inverse_rmse (the inverse's own row index);
    "rows": wc_forward_rows + wc_inverse_rows (the forward writes the unit's
    2 095 105-entry row index, read by the inverse: the round-trip form)."""
    import torch
    cs = CASES[name]
    (w, h, d), (W, H, D) = cs["small"], cs["big"]
    n_cells = W * H * D
    assert n_cells <= 2 ** 31 - 1
    b64 = oracle.synth_box_f64(oracle.unit_seed(cs["seed"], 0, 0, 0), (0, 0, 0), w, h, d)
    b32 = oracle.narrow(b64)
    ex = TiledExpect(oracle, b32, KEEP)
    dev = torch.device("cuda", 0)
    src = b64 if cs["dtype"] == np.float64 else b32
    code = wc.capi.WC_F64 if cs["dtype"] == np.float64 else wc.capi.WC_F32
    cells = ex.tiled(torch, src, dev, W, H, D)
    units, n, extent = wc.capi.make_units([(W, H, D)])
    cap = wc.capi.payload_bound(units, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    regen = torch.full((extent,), float("nan"), dtype=torch.float32, device=dev)
    rmse = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()  # torch's fills ran on its own stream
    if path == "rows":
        rb = wc.capi.rowindex_bytes(units, n)
        assert rb == 8 * (W * H + 1)
        rows = torch.empty(rb // 8, dtype=torch.int64, device=dev)
        torch.cuda.synchronize()
        ctx.forward_rows(cells.data_ptr(), code, units, n, KEEP, payload.data_ptr(), cap, offsets.data_ptr(),
                         kept.data_ptr(), rows.data_ptr(), rb)
        ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, rows.data_ptr(), regen.data_ptr(),
                         cells.data_ptr(), code, rmse.data_ptr())
    else:
        ctx.forward(cells.data_ptr(), code, units, n, KEEP, payload.data_ptr(), cap, offsets.data_ptr(),
                    kept.data_ptr())
        ctx.inverse_rmse(payload.data_ptr(), offsets.data_ptr(), units, n, cells.data_ptr(), code,
                         regen.data_ptr(), rmse.data_ptr())
    ctx.synchronize()
    del cells
    if path == "rows":
        # the sentinel entry (W*H): (nrle, ncoeff - W*H*D = 0)
        assert rows[W * H:W * H + 1].view(torch.int32).tolist() == [int(kept[0]), 0]
        del rows
    tiles = (W // w) * (H // h) * (D // d)
    k = int(kept[0])
    assert k == ex.kept * tiles
    off = offsets.cpu().numpy()
    assert off[0] == 4 and off[1] == 4 + 20 + 8 * k
    hdr = payload[4:24].cpu().numpy().view("<i4")
    assert hdr.tolist() == [W, H, D, n_cells, k]
    pairs = payload[24:24 + 8 * k].view(torch.int32).reshape(-1, 2)
    at = 0
    for want in ex.pair_slabs(torch, dev, W, H, D):
        got = pairs[at:at + want.shape[0]]
        assert torch.equal(got, want), (name, at)
        at += want.shape[0]
    assert at == k
    del pairs, payload
    r3 = regen.reshape(D, H, W)
    z = 0
    for want in ex.regen_slabs(torch, dev, W, H, D):
        assert torch.equal(r3[z:z + d], want), (name, z)
        z += d
    assert z == D
    assert float(rmse[0]) == pytest.approx(ex.rmse, rel=1e-9)
    del regen, r3
    torch.cuda.empty_cache()


def test_more_than_int32_cells_rejected(wc, ctx):
    """2048 x 1024 x 1024 = 2^31 cells: ncoeff would not fit the header's int32."""
    import torch
    units, n, _ = wc.capi.make_units([(2048, 1024, 1024)])
    dev = torch.device("cuda", 0)
    buf = torch.zeros(64, dtype=torch.uint8, device=dev)
    with pytest.raises(wc.WaveletError) as ei:
        ctx.forward(buf.data_ptr(), wc.capi.WC_F32, units, n, KEEP, buf.data_ptr(), 2 ** 40, buf.data_ptr(),
                    buf.data_ptr())
    assert ei.value.code == wc.capi.WC_ERR_INVALID
    with pytest.raises(wc.WaveletError) as ei:
        ctx.inverse(buf.data_ptr(), buf.data_ptr(), units, n, buf.data_ptr())
    assert ei.value.code == wc.capi.WC_ERR_INVALID
