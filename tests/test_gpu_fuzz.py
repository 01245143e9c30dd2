"""Seeded random batches through every device entry point, against the CPU oracle.

The other GPU tests pin chosen shapes, the bench workloads at full size and
the special boxes one by one; this one mixes them the way a caller's batch
would: random dims (odd and even, thin and cubic, sizes that land on the
specialised, fast, generic and sparse-staging paths), random cell offsets
(aligned and not), random fields per unit (the smooth SURVEY field, wide-range
Gaussians, constants of either sign, all-zero, subnormals, NaN / inf
sprinkled in), one random float32 keep per batch (the reference's Config::keep,
src/argparse.h:13), fp64 and fp32 cells.  Per batch:

  * wc_forward: every payload = oracle compress() minus xz
    (src/compressor.cpp:192-248);
  * wc_forward_rows + wc_inverse_rows with the fused RMSE: the same payloads;
    every reconstruction = oracle decompress() (src/decompressor.cpp:238-255)
    bit for bit, a NaN matching any NaN (same_cells); every RMSE = calc_rmse_per_box (src/calc-loss.cpp:12-43)
    within max(1e-12, (n + 4) 2^-53) relative for a box of n cells (NaN where
    the oracle's is NaN).  Both sides add the same n exact double terms (a
    float difference squared in double is exact); only the order differs (the
    reference sums in z, y, x order, the GPU per tile then tiles in order), so
    each sum is within (n - 1) 2^-53 of the exact one and the square root halves
    that; the 1e-12 floor holds for the smooth fields, and the wide-range
    Gaussian fields (ten to the +-30) reach ~1e-12 on 10^5-10^6-cell boxes
    (seed 56 of a 300-seed soak: 1.02e-12 on a 128 x 64 x 96 box);
  * wc_inverse from the payloads alone: the same reconstructions.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = (1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 15, 16, 17, 24, 31, 32, 33, 40, 48, 63, 64)
# WC_FUZZ_SEEDS=N: N seeds per test instead of the suite's 6 / 4 (a longer soak; seeds >= the
# defaults draw batches the default suite does not)
_N = int(os.environ.get("WC_FUZZ_SEEDS", "0"))


def same_cells(got, want):
    """Bit for bit, except that a NaN matches any NaN: IEEE 754 does not specify
    the sign or payload of a NaN result, and the reference's own depend on its
    compiler (which operand of a double addition it keeps; DESIGN.md "Numerics").
    Payload bytes never hold a NaN (a NaN coefficient is never kept)."""
    g, w = np.asarray(got, np.float32), np.asarray(want, np.float32)
    gn, wn = np.isnan(g), np.isnan(w)
    return g.shape == w.shape and np.array_equal(gn, wn) and g[~gn].tobytes() == w[~wn].tobytes()


def _dims(rng, n):
    out = []
    for _ in range(n):
        if rng.random() < 0.1:  # a few large, specialised-shape boxes
            out.append(tuple(int(x) for x in rng.choice([64, 96, 128], size=3)))
        else:
            out.append(tuple(int(x) for x in rng.choice(SIZES, size=3)))
    return out


def _field(rng, O, i, dims):
    W, H, D = dims
    kind = rng.integers(0, 8)
    if kind <= 2:  # the SURVEY §8(d) field
        return O.synth_box_f64(O.unit_seed(99, 1, i, int(kind)), (W * i % 997, 7 * i, 3 * i), W, H, D)
    if kind == 3:  # wide-range Gaussian, mixed sign
        return rng.standard_normal((D, H, W)) * 10.0 ** rng.uniform(-30, 30)
    if kind == 4:  # a constant of either sign (sign quirk: a negative max keeps everything)
        return np.full((D, H, W), rng.choice([-1.0, 1.0]) * rng.uniform(0.1, 1e3))
    if kind == 5:  # all zero
        return np.zeros((D, H, W))
    if kind == 6:  # subnormal-scale values (fp32 denormals survive: no FTZ)
        return rng.standard_normal((D, H, W)) * 1e-41
    b = rng.standard_normal((D, H, W)) * 100.0  # specials sprinkled in
    flat = b.reshape(-1)
    for v in (np.nan, np.inf, -np.inf, 0.0, -0.0):
        if flat.size and rng.random() < 0.5:
            flat[rng.integers(0, flat.size)] = v
    return b


def _batch(O, seed):
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(20, 120))
    dims = _dims(rng, n)
    boxes = [_field(rng, O, i, d) for i, d in enumerate(dims)]
    dtype = np.float64 if seed % 2 == 0 else np.float32
    # cell offsets: packed with random gaps, every third unit at an odd element offset
    offs, cur = [], 0
    for i, (W, H, D) in enumerate(dims):
        cur += int(rng.integers(0, 9))
        if i % 3 == 0 and cur % 2 == 0:
            cur += 1
        offs.append(cur)
        cur += W * H * D
    keep = float(np.float32(rng.choice([rng.uniform(0.5, 0.99999), 0.999, 0.0, 1.0, 1.5])))
    return boxes, dims, offs, cur, dtype, keep


@pytest.mark.parametrize("seed", range(_N or 6))
def test_random_batch_all_entry_points(wc, ctx, oracle, seed):
    _check_all_entry_points(wc, ctx, oracle, seed, seed)


# Library options every path must produce the same bytes under (include/wavelet_amd.h
# wc_set_option): dense staging, the ticket look-back, the worst dispatch order, a wait bound
# of one poll (every look-back wait derives its predecessor), both of those, the dense-decode
# inverse.
_OPTION_SETS = {
    "dense_staging": (("WC_OPT_SPARSE", 0),),
    "tickets": (("WC_OPT_TICKETS", 1),),
    "reversed_tiles": (("WC_OPT_REVERSE_TILES", 1),),
    "spin_limit_1": (("WC_OPT_SPIN_LIMIT", 1),),
    "reversed_spin_1": (("WC_OPT_REVERSE_TILES", 1), ("WC_OPT_SPIN_LIMIT", 1)),
    "dense_inverse": (("WC_OPT_INVERSE_ROWS", 0),),
}


@pytest.mark.parametrize("seed", range(_N or 2))
@pytest.mark.parametrize("opts", sorted(_OPTION_SETS))
def test_random_batch_option_paths(wc, ctx, oracle, seed, opts):
    """The random batches above through every entry point with each option set of
    _OPTION_SETS: payloads, reconstructions and RMSEs as with the defaults (the
    oracle's), the options restored afterwards."""
    keys = [(getattr(wc.capi, name), v) for name, v in _OPTION_SETS[opts]]
    before = [(k, ctx.get_option(k)) for k, _ in keys]
    for k, v in keys:
        ctx.set_option(k, v)
    try:
        _check_all_entry_points(wc, ctx, oracle, 20 + seed, (opts, seed))
    finally:
        for k, v in before:
            ctx.set_option(k, v)


def _check_all_entry_points(wc, ctx, oracle, batch_seed, seed):
    import torch
    boxes, dims, offs, extent, dtype, keep = _batch(oracle, batch_seed)
    units, n, ext = wc.capi.make_units(dims, offsets=offs)
    assert ext == extent
    host = np.zeros(max(extent, 1), dtype)
    for o, b in zip(offs, boxes):
        host[o:o + b.size] = b.ravel().astype(dtype)
    code = wc.capi.WC_F64 if dtype == np.float64 else wc.capi.WC_F32
    dev = torch.device("cuda", 0)
    cells = torch.from_numpy(host).to(dev)
    cap = wc.capi.payload_bound(units, n)
    rb = wc.capi.rowindex_bytes(units, n)

    def bufs():
        return (torch.zeros(cap, dtype=torch.uint8, device=dev), torch.zeros(n + 1, dtype=torch.int64, device=dev),
                torch.zeros(n, dtype=torch.int32, device=dev))

    pay, po, kept = bufs()
    pay2, po2, kept2 = bufs()
    rows = torch.zeros(max(rb // 8, 1), dtype=torch.int64, device=dev)
    out = torch.full((max(extent, 1),), float("nan"), dtype=torch.float32, device=dev)
    out2 = torch.full((max(extent, 1),), float("nan"), dtype=torch.float32, device=dev)
    rmse = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.forward(cells.data_ptr(), code, units, n, keep, pay.data_ptr(), cap, po.data_ptr(), kept.data_ptr())
    ctx.forward_rows(cells.data_ptr(), code, units, n, keep, pay2.data_ptr(), cap, po2.data_ptr(), kept2.data_ptr(),
                     rows.data_ptr(), rb)
    ctx.inverse_rows(pay2.data_ptr(), po2.data_ptr(), units, n, rows.data_ptr(), out.data_ptr(), cells.data_ptr(),
                     code, rmse.data_ptr())
    ctx.inverse(pay.data_ptr(), po.data_ptr(), units, n, out2.data_ptr())
    ctx.synchronize()
    P, O_, K = pay.cpu().numpy(), po.cpu().numpy(), kept.cpu().numpy()
    assert np.array_equal(O_, po2.cpu().numpy()) and np.array_equal(K, kept2.cpu().numpy())
    P2 = pay2.cpu().numpy()
    R, R2, E = out.cpu().numpy(), out2.cpu().numpy(), rmse.cpu().numpy()
    for i, b in enumerate(boxes):
        b32 = oracle.narrow(b) if dtype == np.float64 else b.astype(np.float32)
        want, wk = oracle.compress_payload(b32, keep)
        a = int(O_[i])
        got = P[a:a + 20 + 8 * int(K[i])].tobytes()
        assert got == want and int(K[i]) == wk, (seed, i, dims[i], keep)
        assert P2[a:a + len(want)].tobytes() == want, (seed, i, "forward_rows")
        if b.size == 0:
            continue
        back = oracle.decompress_payload(want).ravel()
        o = offs[i]
        assert same_cells(R[o:o + b.size], back), (seed, i, dims[i], "inverse_rows")
        assert same_cells(R2[o:o + b.size], back), (seed, i, dims[i], "inverse")
        ref = oracle.rmse(b32, back.reshape(b32.shape))
        if np.isnan(ref):
            assert np.isnan(E[i]), (seed, i, E[i])
        elif np.isinf(ref):
            assert E[i] == ref, (seed, i, E[i], ref)
        else:
            tol = max(1e-12, (b.size + 4) * 2.0 ** -53)
            assert abs(E[i] - ref) <= tol * abs(ref), (seed, i, dims[i], E[i], ref)


@pytest.mark.parametrize("seed", range(_N or 4))
def test_random_batch_global_threshold_mode(wc, ctx, oracle, seed):
    """The opt-in global-threshold mode on the same random batches: the
    histogram (counted inside K1 for the fast units, by k_hist for the generic
    ones) equals the oracle's bins, and the payloads at the thresholds of three
    quantiles equal the reference's mask + RLE + serialize at that threshold."""
    import torch
    boxes, dims, offs, extent, dtype, _ = _batch(oracle, seed + 10)
    units, n, _ = wc.capi.make_units(dims, offsets=offs)
    host = np.zeros(max(extent, 1), dtype)
    for o, b in zip(offs, boxes):
        host[o:o + b.size] = b.ravel().astype(dtype)
    code = wc.capi.WC_F64 if dtype == np.float64 else wc.capi.WC_F32
    dev = torch.device("cuda", 0)
    cells = torch.from_numpy(host).to(dev)
    cap = wc.capi.payload_bound(units, n)
    hist = torch.zeros(wc.capi.HIST_BINS, dtype=torch.int64, device=dev)
    pay = torch.zeros(cap, dtype=torch.uint8, device=dev)
    po = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.forward_stage(cells.data_ptr(), code, units, n, hist.data_ptr())
    ctx.synchronize()
    h = hist.cpu().numpy().view(np.uint64)
    b32 = [oracle.narrow(b) if dtype == np.float64 else b.astype(np.float32) for b in boxes]
    with np.errstate(all="ignore"):
        want = sum(oracle.magnitude_hist(oracle.wavelet_decompose(b)) for b in b32)
    assert np.array_equal(h, want), seed
    for q in (0.3, 0.9, 0.999):
        t, r = wc.capi.hist_threshold(h, q)
        ctx.forward_emit(units, n, 0.0, t, pay.data_ptr(), cap, po.data_ptr(), kept.data_ptr())
        ctx.synchronize()
        P, O_, K = pay.cpu().numpy(), po.cpu().numpy(), kept.cpu().numpy()
        assert int(K.astype(np.int64).sum()) == r, (seed, q)
        for i, b in enumerate(b32):
            a = int(O_[i])
            assert P[a:a + 20 + 8 * int(K[i])].tobytes() == oracle.compress_payload_thresh(b, t), (seed, q, i, dims[i])


@pytest.mark.parametrize("seed", range(_N or 3))
def test_random_batch_host_entry_points(wc, ctx, oracle, seed):
    """The random batches through the host-buffer entry points (PCIe-inclusive;
    include/wavelet_amd.h wc_forward_host, wc_forward_host_units,
    wc_round_trip_host, wc_inverse_host) with a random pipelined unit-run size
    (WC_OPT_HOST_CHUNK: one run, or runs of 2^14 .. 2^25 cells): densely packed
    payloads equal to the oracle's compress() minus xz, reconstructions equal to
    its decompress(), RMSEs within the summation-order bound."""
    boxes, dims, offs, extent, dtype, keep = _batch(oracle, 40 + seed)
    units, n, ext = wc.capi.make_units(dims, offsets=offs)
    host = np.zeros(max(extent, 1), dtype)
    for o, b in zip(offs, boxes):
        host[o:o + b.size] = b.ravel().astype(dtype)
    chunk = int(np.random.default_rng(seed).choice([0, 1 << 14, 1 << 18, 1 << 21, 1 << 25]))
    before = ctx.get_option(wc.capi.WC_OPT_HOST_CHUNK)
    ctx.set_option(wc.capi.WC_OPT_HOST_CHUNK, chunk)
    try:
        pay, po, kept = ctx.forward_host(host, units, n, keep)
        pay_u, po_u, kept_u = ctx.forward_host_units([host[o:o + b.size] for o, b in zip(offs, boxes)], units, n,
                                                     keep)
        pay_r, po_r, kept_r, rmse = ctx.round_trip_host(host, units, n, keep)
        regen = ctx.inverse_host(pay, po, units, n, extent)
    finally:
        ctx.set_option(wc.capi.WC_OPT_HOST_CHUNK, before)
    for i, b in enumerate(boxes):
        b32 = oracle.narrow(b) if dtype == np.float64 else b.astype(np.float32)
        want, wk = oracle.compress_payload(b32, keep)
        for tag, (p, o, k) in (("forward_host", (pay, po, kept)), ("forward_host_units", (pay_u, po_u, kept_u)),
                               ("round_trip_host", (pay_r, po_r, kept_r))):
            assert wc.capi.unit_payload(p, o, k, i) == want and int(k[i]) == wk, (seed, chunk, i, dims[i], tag)
        if b.size == 0:
            continue
        back = oracle.decompress_payload(want).ravel()
        assert same_cells(regen[offs[i]:offs[i] + b.size], back), (seed, chunk, i, dims[i], "inverse_host")
        ref = oracle.rmse(b32, back.reshape(b32.shape))
        if np.isnan(ref):
            assert np.isnan(rmse[i]), (seed, i, rmse[i])
        elif np.isinf(ref):
            assert rmse[i] == ref, (seed, i, rmse[i], ref)
        else:
            tol = max(1e-12, (b.size + 4) * 2.0 ** -53)
            assert abs(rmse[i] - ref) <= tol * abs(ref), (seed, chunk, i, dims[i], rmse[i], ref)


@pytest.mark.parametrize("seed", range(_N or 4))
def test_random_boxes_python_mirror(wc, oracle, seed, tmp_path):
    """Seeded random multiBox3Ds (1-4 float32 components of one random shape, the
    fields of _field) through the Python mirror of the reference API
    (wavelet-compression_amd/codec.py): compress() (src/compressor.cpp:192-297)
    returns the oracle's pairs and writes the .xz files under the reference's
    names (:250-254); decompress() of each file (src/decompressor.cpp:238-255),
    wavelet_decompose -> inverse_wavelet_decompose of the box, and
    calc_rmse_per_box (src/calc-loss.cpp:12-43) agree with the oracle (a NaN
    matching any NaN; the RMSE within the summation-order bound)."""
    from wavelet_compression_amd import codec
    rng = np.random.default_rng(5000 + seed)
    W, H, D = (int(x) for x in rng.choice(SIZES, size=3))
    ncomp = int(rng.integers(1, 5))
    boxes = [_field(rng, oracle, i, (W, H, D)).astype(np.float32) for i in range(ncomp)]
    comps = [int(c) for c in rng.choice(40, size=ncomp, replace=False)]
    keep = float(np.float32(rng.choice([rng.uniform(0.5, 0.99999), 0.999, 0.0, 1.0, 1.5])))
    t, lev, bi = int(rng.integers(0, 10)), int(rng.integers(0, 4)), int(rng.integers(0, 1000))
    with np.errstate(all="ignore"):
        cws = codec.compress(boxes, comps, keep, t, lev, bi, tmp_path)
        assert len(cws) == ncomp
        regen = []
        for c, b in enumerate(boxes):
            want, wk = oracle.compress_payload(b, keep)
            assert codec.serialize_compressed_wavelet(cws[c]) == want and len(cws[c].rle_encoded) == wk, (seed, c)
            f = tmp_path / f"compressed-wavelet-{t}-{lev}-{comps[c]}-{bi}.xz"
            assert f.exists(), f
            back = oracle.decompress_payload(want)
            r = codec.decompress(f)
            assert r.shape == (D, H, W) and same_cells(r.ravel(), back.ravel()), (seed, c, (W, H, D), keep)
            flat = codec.wavelet_decompose(b)
            assert same_cells(flat, oracle.wavelet_decompose(b)), (seed, c, "wavelet_decompose")
            assert same_cells(codec.inverse_wavelet_decompose(flat, W, H, D).ravel(),
                              oracle.inverse_wavelet_decompose(flat, W, H, D).ravel()), (seed, c, "inverse")
            regen.append(r)
        rm = codec.calc_rmse_per_box(regen, boxes, ncomp)
        for c in range(ncomp):
            ref = oracle.rmse(regen[c], boxes[c])
            if np.isnan(ref):
                assert np.isnan(rm[c]), (seed, c)
            elif np.isinf(ref):
                assert rm[c] == ref, (seed, c)
            else:
                tol = max(1e-12, (W * H * D + 4) * 2.0 ** -53)
                assert abs(rm[c] - ref) <= tol * abs(ref), (seed, c, rm[c], ref)
