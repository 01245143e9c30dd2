"""GPU parity of the in-process round trip (include/wavelet_amd.h wc_forward_rows
+ wc_inverse_rows): the forward writes each payload's row index as it packs the
pairs, the inverse reads it instead of running the row index kernel.

The reference's -estimate compresses and decompresses the same boxes
(src/modes.cpp:236-291: compress(), decompress() = rle_decode +
inverse_wavelet_decompose, src/decompressor.cpp:14-159, calc_rmse_per_box,
src/calc-loss.cpp:12-43); the bar is the same as the two-call path:
  * payloads, offsets and kept counts byte-identical to wc_forward's (and so to
    the oracle's, tests/test_gpu_parity.py);
  * the row index equal, entry for entry, to the numpy restatement derived
    from the payload (tests/numpy_ref.py row_index);
  * reconstructions bit-exact against the oracle's decompress(), RMSE within
    1e-12 of calc_rmse_per_box;
  * over every shape class: the fast (row-indexed) shapes, odd shapes (dense
    decode beside them), empty units, all-zero units (only trailing rows),
    sparse units (long gaps: a pair opens many rows), NaN-first units
    (nothing kept), the ticket form of the look-backs;
  * a row index that does not belong to the payloads gives wrong cells but no
    fault; a header that disagrees with its unit is WC_ERR_FORMAT;
  * fp64 originals at a base that is not 16-B aligned (the separate RMSE pass).
"""
import numpy as np
import pytest

import numpy_ref as R
from test_gpu_parity import DIMS, KEEPS, synth
from wavelet_compression_amd.capi import WC_OPT_ORDERED, WaveletError

pytestmark = pytest.mark.gpu


def _special():
    out = []
    out.append(np.zeros((8, 4, 6), np.float32))                      # all zero: trailing rows only
    b = np.zeros((32, 16, 16), np.float32); b[20, 3, 5] = 7.0        # one spike: long gaps both sides
    out.append(b)
    b = np.full((16, 8, 8), 2.0, np.float32); b[:2, :2, :2] = np.nan  # NaN first: nothing kept
    out.append(b)
    b = np.full((64, 32, 32), 5.0, np.float32); b[63, 31, 31] = 9.0  # the last coefficient block only
    out.append(b)
    out.append(np.zeros((0, 4, 4), np.float32))                      # empty unit
    b = (np.random.default_rng(3).standard_normal((64, 64, 64)) * 0.001).astype(np.float32)
    b[::7, ::5, ::3] += 40.0                                         # scattered spikes, keep 0.5: sparse
    out.append(b)
    return out


def _device_batch(wc, boxes, dtype=np.float64):
    import torch
    dims = [(b.shape[2], b.shape[1], b.shape[0]) for b in boxes]
    units, n, extent = wc.capi.make_units(dims)
    cells = np.zeros(max(extent, 1), dtype)
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        cells[o:o + b.size] = b.ravel().astype(dtype)
    dev = torch.device("cuda", 0)
    return units, n, extent, torch.from_numpy(cells).to(dev), dev


def _round_trip(wc, ctx, boxes, keep, dtype=np.float64, rows=True):
    """wc_forward_rows + wc_inverse_rows (rows) or wc_forward + wc_inverse_rmse."""
    import torch
    units, n, extent, d_cells, dev = _device_batch(wc, boxes, dtype)
    code = wc.capi.WC_F64 if dtype == np.float64 else wc.capi.WC_F32
    cap = wc.capi.payload_bound(units, n)
    rb = wc.capi.rowindex_bytes(units, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(max(n, 1), dtype=torch.int32, device=dev)
    rowinfo = torch.full((rb // 4,), 0xA5A5A5A5 - (1 << 32), dtype=torch.int32, device=dev)
    regen = torch.full((max(extent, 1),), float("nan"), dtype=torch.float32, device=dev)
    rmse = torch.full((max(n, 1),), -1.0, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    if rows:
        ctx.forward_rows(d_cells.data_ptr(), code, units, n, keep, payload.data_ptr(), cap, offsets.data_ptr(),
                         kept.data_ptr(), rowinfo.data_ptr(), rb)
        ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, rowinfo.data_ptr(), regen.data_ptr(),
                         d_cells.data_ptr(), code, rmse.data_ptr())
    else:
        ctx.forward(d_cells.data_ptr(), code, units, n, keep, payload.data_ptr(), cap, offsets.data_ptr(),
                    kept.data_ptr())
        ctx.inverse_rmse(payload.data_ptr(), offsets.data_ptr(), units, n, d_cells.data_ptr(), code,
                         regen.data_ptr(), rmse.data_ptr())
    ctx.synchronize()
    return dict(units=units, n=n, payload=payload.cpu().numpy(), offsets=offsets.cpu().numpy(),
                kept=kept.cpu().numpy()[:n], rowinfo=rowinfo.cpu().numpy().view(np.uint32).reshape(-1, 2),
                regen=regen.cpu().numpy(), rmse=rmse.cpu().numpy()[:n])


def _check(oracle, boxes, r, keep):
    ent = 0
    for i, b in enumerate(boxes):
        u = r["units"][i]
        W, H, D = u.nx, u.ny, u.nz
        b32 = oracle.narrow(b) if b.dtype == np.float64 else b
        want, k = oracle.compress_payload(b32, keep)
        po = int(r["offsets"][i])
        got = r["payload"][po:po + 20 + 8 * int(r["kept"][i])].tobytes()
        assert got == want and int(r["kept"][i]) == k, (i, (W, H, D))
        if b.size:
            back = oracle.decompress_payload(want)
            o = u.cell_offset
            assert r["regen"][o:o + b.size].tobytes() == back.ravel().tobytes(), (i, (W, H, D))
            ref = oracle.rmse(b32, back)
            if np.isnan(ref):  # NaN cells: NaN RMSE, as calc_rmse_per_box's sum
                assert np.isnan(r["rmse"][i]), (i, r["rmse"][i])
            else:
                assert abs(r["rmse"][i] - ref) <= 1e-12 * abs(ref), (i, r["rmse"][i], ref)
        fast = b.size > 0 and W % 2 == 0 and H % 2 == 0 and D % 8 == 0
        if fast:  # the forward wrote the unit's row index: every entry as the restatement derives it
            assert np.array_equal(r["rowinfo"][ent:ent + W * H + 1], R.row_index(want, W, H, D)), (i, (W, H, D))
        if b.size:  # an empty unit owns no row-index entries (wc_rowindex_bytes)
            ent += W * H + 1


@pytest.mark.parametrize("keep", KEEPS)
def test_round_trip_rows_shapes(wc, ctx, oracle, keep):
    boxes = synth(oracle, DIMS, seed0=11)
    _check(oracle, boxes, _round_trip(wc, ctx, boxes, keep), keep)


@pytest.mark.parametrize("ordered", [1, 0])
def test_round_trip_rows_special(wc, ctx, oracle, ordered):
    boxes = _special()
    keep = float(np.float32(0.5))
    ctx.set_option(WC_OPT_ORDERED, ordered)
    try:
        r = _round_trip(wc, ctx, boxes, keep, dtype=np.float32)
    finally:
        ctx.set_option(WC_OPT_ORDERED, 1)
    _check(oracle, boxes, r, keep)


def test_round_trip_rows_equals_two_call_path(wc, ctx, oracle):
    """Same bytes, cells and RMSE as wc_forward + wc_inverse_rmse (fp32 cells,
    the drop-in compress() input type)."""
    boxes = [oracle.narrow(b) for b in synth(oracle, [(64, 64, 64)] * 6 + [(32, 32, 32)] * 8 + DIMS, seed0=12)]
    keep = KEEPS[1]
    a = _round_trip(wc, ctx, boxes, keep, np.float32, rows=True)
    b = _round_trip(wc, ctx, boxes, keep, np.float32, rows=False)
    n = a["n"]
    assert np.array_equal(a["offsets"], b["offsets"]) and np.array_equal(a["kept"], b["kept"])
    for i in range(n):
        po = int(a["offsets"][i])
        end = po + 20 + 8 * int(a["kept"][i])
        assert np.array_equal(a["payload"][po:end], b["payload"][po:end]), i
    assert a["regen"].tobytes() == b["regen"].tobytes()
    assert np.array_equal(a["rmse"], b["rmse"])  # the same fused sums in the same order
    _check(oracle, boxes, a, keep)


def test_inverse_rows_foreign_row_index_no_fault(wc, ctx, oracle):
    """A row index of other payloads (here: random words) reads only pairs of
    these payloads (entries clamped to each payload's pair count): the call
    completes; the cells are whatever those pairs give."""
    import torch
    boxes = synth(oracle, [(64, 64, 64), (32, 16, 64), (16, 16, 16)], seed0=13)
    keep = KEEPS[1]
    units, n, extent, d_cells, dev = _device_batch(wc, boxes)
    cap = wc.capi.payload_bound(units, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    rb = wc.capi.rowindex_bytes(units, n)
    junk = torch.randint(-(1 << 31), (1 << 31) - 1, (rb // 4,), dtype=torch.int32, device=dev)
    regen = torch.zeros(extent, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    ctx.forward(d_cells.data_ptr(), wc.capi.WC_F64, units, n, keep, payload.data_ptr(), cap, offsets.data_ptr(),
                kept.data_ptr())
    ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, junk.data_ptr(), regen.data_ptr())
    ctx.synchronize()
    # the same payloads with their own row index (from the payloads) are exact again
    ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, None, regen.data_ptr())
    ctx.synchronize()
    got = regen.cpu().numpy()
    for i, b in enumerate(boxes):
        want = oracle.decompress_payload(oracle.compress_payload(oracle.narrow(b), keep)[0])
        o = units[i].cell_offset
        assert got[o:o + b.size].tobytes() == want.ravel().tobytes(), i


def test_inverse_rows_bad_header_is_format_error(wc, ctx, oracle):
    import torch
    boxes = synth(oracle, [(16, 16, 16), (32, 32, 32)], seed0=14)
    keep = KEEPS[1]
    units, n, extent, d_cells, dev = _device_batch(wc, boxes)
    cap = wc.capi.payload_bound(units, n)
    rb = wc.capi.rowindex_bytes(units, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    rowinfo = torch.zeros(rb // 4, dtype=torch.int32, device=dev)
    regen = torch.zeros(extent, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    ctx.forward_rows(d_cells.data_ptr(), wc.capi.WC_F64, units, n, keep, payload.data_ptr(), cap,
                     offsets.data_ptr(), kept.data_ptr(), rowinfo.data_ptr(), rb)
    ctx.synchronize()
    po = int(offsets[1].item())
    payload[po:po + 4] = torch.tensor(np.array([33], "<i4").view(np.uint8), device=dev)  # W 32 -> 33
    torch.cuda.synchronize()
    ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, rowinfo.data_ptr(), regen.data_ptr())
    with pytest.raises(WaveletError) as e:
        ctx.synchronize()
    assert e.value.code == wc.capi.WC_ERR_FORMAT
    # the context is usable afterwards
    payload[po:po + 4] = torch.tensor(np.array([32], "<i4").view(np.uint8), device=dev)
    torch.cuda.synchronize()
    ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, rowinfo.data_ptr(), regen.data_ptr())
    ctx.synchronize()


def test_rmse_unaligned_fp64_originals(wc, ctx, oracle):
    """fp64 originals at a base 8 bytes past a 16-B boundary: the fused inverse
    takes the separate RMSE pass (no 16-B loads there); same RMSE as aligned."""
    import torch
    boxes = synth(oracle, [(64, 64, 64), (32, 32, 32), (16, 16, 16)], seed0=15)
    keep = KEEPS[1]
    units, n, extent, d_cells, dev = _device_batch(wc, boxes)
    cap = wc.capi.payload_bound(units, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    regen = torch.zeros(extent, dtype=torch.float32, device=dev)
    shifted = torch.zeros(extent + 1, dtype=torch.float64, device=dev)
    shifted[1:] = d_cells
    r_al = torch.zeros(n, dtype=torch.float64, device=dev)
    r_un = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.forward(d_cells.data_ptr(), wc.capi.WC_F64, units, n, keep, payload.data_ptr(), cap, offsets.data_ptr(),
                kept.data_ptr())
    ctx.inverse_rmse(payload.data_ptr(), offsets.data_ptr(), units, n, d_cells.data_ptr(), wc.capi.WC_F64,
                     regen.data_ptr(), r_al.data_ptr())
    assert (shifted[1:].data_ptr() & 15) == 8
    ctx.inverse_rmse(payload.data_ptr(), offsets.data_ptr(), units, n, shifted[1:].data_ptr(), wc.capi.WC_F64,
                     regen.data_ptr(), r_un.data_ptr())
    ctx.synchronize()
    a, u = r_al.cpu().numpy(), r_un.cpu().numpy()
    for i, b in enumerate(boxes):
        want = oracle.rmse(oracle.narrow(b), regen.cpu().numpy()[units[i].cell_offset:][:b.size].reshape(b.shape))
        assert abs(u[i] - want) <= 1e-12 * want and abs(a[i] - want) <= 1e-12 * want, i


def test_misaligned_device_buffers_rejected(wc, ctx):
    import torch
    units, n, extent = wc.capi.make_units([(16, 16, 16)])
    dev = torch.device("cuda", 0)
    cells = torch.zeros(extent + 4, dtype=torch.float32, device=dev)
    cap = wc.capi.payload_bound(units, n)
    payload = torch.zeros(cap + 16, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(WaveletError) as e:
        ctx.forward(cells[1:].data_ptr(), wc.capi.WC_F32, units, n, 0.999, payload.data_ptr(), cap,
                    offsets.data_ptr(), kept.data_ptr())
    assert e.value.code == wc.capi.WC_ERR_INVALID and "aligned" in str(e.value)
    with pytest.raises(WaveletError):
        ctx.forward(cells.data_ptr(), wc.capi.WC_F32, units, n, 0.999, payload[4:].data_ptr(), cap,
                    offsets.data_ptr(), kept.data_ptr())
    with pytest.raises(WaveletError):
        ctx.inverse(payload.data_ptr(), offsets.data_ptr(), units, n, cells[2:].data_ptr())


def test_row_index_capacity_checked(wc, ctx, oracle):
    """A row index buffer smaller than wc_rowindex_bytes is rejected by both
    calls (WC_ERR_INVALID before any launch), never read or written past."""
    import torch
    boxes = synth(oracle, [(16, 16, 16), (32, 16, 8)], seed0=19)
    units, n, extent, d_cells, dev = _device_batch(wc, boxes)
    cap = wc.capi.payload_bound(units, n)
    rb = wc.capi.rowindex_bytes(units, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    rows = torch.zeros(rb // 8, dtype=torch.int64, device=dev)
    out = torch.zeros(extent, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    with pytest.raises(WaveletError) as e:
        ctx.forward_rows(d_cells.data_ptr(), wc.capi.WC_F64, units, n, 0.999, payload.data_ptr(), cap,
                         offsets.data_ptr(), kept.data_ptr(), rows.data_ptr(), rb - 8)
    assert e.value.code == wc.capi.WC_ERR_INVALID
    ctx.forward_rows(d_cells.data_ptr(), wc.capi.WC_F64, units, n, 0.999, payload.data_ptr(), cap,
                     offsets.data_ptr(), kept.data_ptr(), rows.data_ptr(), rb)
    with pytest.raises(WaveletError) as e:
        ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, rows.data_ptr(), out.data_ptr(),
                         rowinfo_capacity=rb - 8)
    assert e.value.code == wc.capi.WC_ERR_INVALID and "rowinfo_capacity" in str(e.value)
    ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), units, n, rows.data_ptr(), out.data_ptr(),
                     rowinfo_capacity=rb)
    ctx.synchronize()


def test_forward_host_units_equals_forward_host(wc, ctx, oracle):
    """wc_forward_host_units (each unit's cells at its own host pointer, the
    drop-in compress()'s call) gives the bytes of wc_forward_host over the
    packed units, and the oracle's."""
    boxes = [oracle.narrow(b) for b in synth(oracle, DIMS + [(64, 64, 64)] * 3, seed0=16)]
    keep = KEEPS[1]
    dims = [(b.shape[2], b.shape[1], b.shape[0]) for b in boxes]
    units, n, extent = wc.capi.make_units(dims)
    cells = np.zeros(max(extent, 1), np.float32)
    for i, b in enumerate(boxes):
        cells[units[i].cell_offset:units[i].cell_offset + b.size] = b.ravel()
    pa, oa, ka = ctx.forward_host(cells, units, n, keep)
    pb, ob, kb = ctx.forward_host_units(boxes, units, n, keep)
    assert np.array_equal(oa, ob) and np.array_equal(ka, kb)
    bad = [(i, wc.capi.unit_payload(pa, oa, ka, i) == oracle.compress_payload(b, keep)[0],
            wc.capi.unit_payload(pb, ob, kb, i) == oracle.compress_payload(b, keep)[0])
           for i, b in enumerate(boxes)
           if wc.capi.unit_payload(pa, oa, ka, i) != wc.capi.unit_payload(pb, ob, kb, i)]
    assert not bad, f"(unit, packed == oracle, per-unit == oracle): {bad}; dims {dims}"
    # bytes [0, offsets[0]) are not written (the first slot starts at 4 mod 8)
    assert np.array_equal(pa[int(oa[0]):int(oa[n])], pb[int(ob[0]):int(ob[n])])
    for i, b in enumerate(boxes):
        assert wc.capi.unit_payload(pb, ob, kb, i) == oracle.compress_payload(b, keep)[0], i


@pytest.mark.parametrize("chunk", [0, 1 << 16])
def test_round_trip_host_runs(wc, ctx, oracle, chunk):
    """wc_round_trip_host (the CLI's -estimate): host cells in, payloads and the
    per-unit RMSE out, the reconstruction never leaving the device; as one run
    (chunk 0) and as pipelined unit runs of 2^16 cells (each run's forward
    writes its row index, its inverse reads it).  Payloads equal the oracle's,
    RMSE within 1e-12 of calc_rmse_per_box on the oracle's reconstruction."""
    from test_gpu_parity import pack
    from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK
    boxes = synth(oracle, DIMS + [(64, 64, 64)] * 6 + [(32, 32, 32)] * 12, seed0=17)
    keep = KEEPS[1]
    units, n, extent, cells = pack(wc, boxes)
    before = ctx.get_option(WC_OPT_HOST_CHUNK)
    ctx.set_option(WC_OPT_HOST_CHUNK, chunk)
    try:
        payload, offs, kept, rmse = ctx.round_trip_host(cells, units, n, keep)
    finally:
        ctx.set_option(WC_OPT_HOST_CHUNK, before)
    for i, b in enumerate(boxes):
        b32 = oracle.narrow(b)
        want = oracle.compress_payload(b32, keep)[0]
        assert wc.capi.unit_payload(payload, offs, kept, i) == want, i
        if b.size:
            ref = oracle.rmse(b32, oracle.decompress_payload(want))
            assert abs(rmse[i] - ref) <= 1e-12 * abs(ref), (i, rmse[i], ref)
