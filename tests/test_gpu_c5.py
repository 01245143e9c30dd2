"""BASELINE.json configs[4] (C5) at full size on one GPU, checked against the
CPU oracle: all 512 x 128^3 fp32 units (bench_workloads.WORKLOADS["c5"]) at
keep 0.9999f in ONE wc_forward (the reference's own loop runs them one by one,
src/compressor.cpp:192-248 per box, src/modes.cpp:100-103):
  * every unit: header (W, H, D, ncoeff, nrle), 0 <= kept <= ncoeff, and the
    worst-case slot offsets;
  * EVERY unit's payload bytes and kept count equal the oracle's compress()
    minus xz (on a 16-thread pool: ctypes releases the GIL);
  * the launch-order and the ticket form of the look-backs write identical
    bytes for ALL 512 units (zeroed payload buffers compared whole);
  * wc_inverse of the whole batch (the c5.inverse leg of bench.py) reproduces
    the oracle's decompress() (rle_decode + inverse_wavelet_decompose,
    src/decompressor.cpp:14-159) bit for bit on ALL 512 units, and so does
    wc_inverse_rows with the row index wc_forward_rows wrote (the payloads of
    which equal wc_forward's).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEEP = float(np.float32(0.9999))


@pytest.fixture(scope="module")
def c5_run(wc, ctx):
    """The session context: the ONLY live context, so the launch-order form
    is the one that runs (a second live context would switch to the tickets)."""
    import torch
    import bench_workloads as bw
    units = bw.WORKLOADS["c5"]["units"]()
    assert len(units) == 512 and all(u.cells == 128 ** 3 for u in units)
    dev = torch.device("cuda", 0)
    cells, offs, extent = bw.synth_cells(torch, dev, units, "f32")
    tab, n, _ = bw.units_array(wc.capi, units, offs)
    cap = wc.capi.payload_bound(tab, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.forward(cells.data_ptr(), wc.capi.WC_F32, tab, n, KEEP, payload.data_ptr(), cap, offsets.data_ptr(),
                kept.data_ptr())
    ctx.synchronize()
    r = dict(units=units, offs=offs, cells=cells, payload=payload, offsets_dev=offsets,
             offsets=offsets.cpu().numpy(), kept=kept.cpu().numpy(), tab=tab, n=n, ctx=ctx, dev=dev, cap=cap,
             extent=extent)
    yield r
    del r, cells, payload
    torch.cuda.empty_cache()


def _host(r, key):
    """One host copy of a device buffer per module (cells: 4 GiB, payload slots: 8.6 GB)."""
    h = r.setdefault("host", {})
    if key not in h:
        h[key] = r[key].cpu().numpy()
    return h[key]


def _payload(r, i):
    po = int(r["offsets"][i])
    return _host(r, "payload")[po:po + 20 + 8 * int(r["kept"][i])].tobytes()


def _threads():
    import os
    return max(1, min(16, os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def test_c5_every_unit_header_kept_and_slots(c5_run):
    import torch
    r = c5_run
    n = r["n"]
    idx = r["offsets_dev"][:n].view(n, 1) + torch.arange(20, device=r["dev"]).view(1, 20)
    hdr = r["payload"][idx.reshape(-1)].cpu().numpy().reshape(n, 20).copy().view("<i4")
    assert np.array_equal(hdr[:, :4], np.tile(np.array([128, 128, 128, 128 ** 3], np.int32), (n, 1)))
    assert np.array_equal(hdr[:, 4], r["kept"].astype(np.int32))
    assert np.all(r["kept"] >= 0) and np.all(r["kept"].astype(np.int64) <= 128 ** 3)
    slots = 4 + np.arange(n, dtype=np.int64) * (24 + 8 * 128 ** 3)
    assert np.array_equal(r["offsets"][:n].astype(np.int64), slots)
    assert int(r["offsets"][n]) == int(slots[-1]) + 20 + 8 * int(r["kept"][-1])
    frac = r["kept"].astype(np.int64).sum() / (n * 128 ** 3)
    assert 0.3 < frac < 0.6  # SURVEY §8(d) field at keep 0.9999: ~45 % kept


def test_c5_every_payload_matches_oracle(c5_run, oracle):
    """All 512 forward payloads (src/compressor.cpp:192-248 per unit, minus xz)
    and kept counts against the oracle, not a sample."""
    from concurrent.futures import ThreadPoolExecutor
    r = c5_run
    cells = _host(r, "cells")

    def check(i):
        u = r["units"][i]
        o = r["offs"][i]
        want, k = oracle.compress_payload(cells[o:o + u.cells].reshape(u.D, u.H, u.W), KEEP)
        return None if (_payload(r, i) == want and int(r["kept"][i]) == k) else i

    with ThreadPoolExecutor(_threads()) as ex:
        bad = [i for i in ex.map(check, range(r["n"])) if i is not None]
    assert not bad, bad[:16]


@pytest.mark.parametrize("ordered", [1, 0])
def test_c5_paths_identical_all_units(c5_run, wc, ordered):
    """The default path's bytes for all 512 units against a second run in the
    launch-order form and in the look-backs' ticket form (WC_OPT_ORDERED 0):
    whole zeroed buffers compared; the option readback shows which form ran."""
    import torch
    from wavelet_compression_amd.capi import WC_OPT_ORDERED
    r = c5_run
    c = r["ctx"]
    other = torch.zeros_like(r["payload"])
    offs = torch.zeros_like(r["offsets_dev"])
    kept = torch.zeros(r["n"], dtype=torch.int32, device=r["dev"])
    # torch filled these on its own stream; the context's stream does not wait
    # for it (round 4: a fill still running zeroed the tail units' kept counts)
    torch.cuda.synchronize()
    try:
        c.set_option(WC_OPT_ORDERED, ordered)
        assert c.get_option(WC_OPT_ORDERED) == ordered
        c.forward(r["cells"].data_ptr(), wc.capi.WC_F32, r["tab"], r["n"], KEEP, other.data_ptr(), r["cap"],
                  offs.data_ptr(), kept.data_ptr())
        c.synchronize()
    finally:
        c.set_option(WC_OPT_ORDERED, 1)
    assert np.array_equal(kept.cpu().numpy(), r["kept"])
    assert np.array_equal(offs.cpu().numpy(), r["offsets"])
    assert torch.equal(other, r["payload"])
    del other
    torch.cuda.empty_cache()


def test_c5_inverse_every_unit_matches_oracle(c5_run, oracle):
    """wc_inverse of all 512 payloads, then wc_forward_rows + wc_inverse_rows:
    every reconstruction equal to the oracle's decompress() of the unit's
    payload (on a 16-thread pool), and the rows forward's payloads equal."""
    import torch
    from concurrent.futures import ThreadPoolExecutor
    r = c5_run
    n = r["n"]
    regen = torch.empty(r["extent"], dtype=torch.float32, device=r["dev"])
    torch.cuda.synchronize()
    r["ctx"].inverse(r["payload"].data_ptr(), r["offsets_dev"].data_ptr(), r["tab"], n, regen.data_ptr())
    r["ctx"].synchronize()
    got = regen.cpu().numpy()

    def check(i):
        want = oracle.decompress_payload(_payload(r, i)).ravel()
        o = r["offs"][i]
        return None if got[o:o + 128 ** 3].tobytes() == want.tobytes() else i

    with ThreadPoolExecutor(_threads()) as ex:
        bad = [i for i in ex.map(check, range(n)) if i is not None]
    assert not bad, bad[:16]

    # the round trip with the forward's row index: same payloads, same cells
    from wavelet_compression_amd.capi import WC_F32, rowindex_bytes
    rb = rowindex_bytes(r["tab"], n)
    rows = torch.empty(rb // 8, dtype=torch.int64, device=r["dev"])
    other = torch.zeros_like(r["payload"])
    offs = torch.zeros_like(r["offsets_dev"])
    kept = torch.zeros(n, dtype=torch.int32, device=r["dev"])
    regen.fill_(float("nan"))
    torch.cuda.synchronize()
    r["ctx"].forward_rows(r["cells"].data_ptr(), WC_F32, r["tab"], n, KEEP, other.data_ptr(), r["cap"],
                          offs.data_ptr(), kept.data_ptr(), rows.data_ptr(), rb)
    r["ctx"].inverse_rows(other.data_ptr(), offs.data_ptr(), r["tab"], n, rows.data_ptr(), regen.data_ptr())
    r["ctx"].synchronize()
    assert torch.equal(other, r["payload"])
    assert regen.cpu().numpy().tobytes() == got.tobytes()
    del regen, rows, other
    torch.cuda.empty_cache()
