"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bar: bit-exact for every integer/byte output (payload bytes => retained index
set, run lengths and values) and for the fp32 transform / reconstruction (the
reference's arithmetic is reproduced exactly); RMSE
within 1e-12 relative (the reference sums sequentially in double, the GPU sums
in a fixed tree order).
"""
import numpy as np
import pytest
from wavelet_compression_amd.capi import WC_OPT_INVERSE_ROWS, WC_OPT_ORDERED, WC_OPT_SPARSE

pytestmark = pytest.mark.gpu

KEEPS = [float(np.float32(k)) for k in (0.99, 0.999, 0.9999)]  # float widened, src/argparse.h:13

DIMS = [
    (2, 2, 2), (8, 4, 2), (6, 10, 14), (3, 4, 2), (3, 5, 7), (1, 1, 1), (1, 7, 1), (5, 1, 9),
    (16, 16, 16), (32, 32, 32), (16, 32, 64), (48, 32, 16), (64, 64, 64), (4, 8, 16),
    (33, 17, 9), (66, 2, 130), (2, 200, 3), (127, 3, 5), (40, 40, 70),
]


def synth(O, dims, seed0=0, sigma=0.05):
    return [O.synth_box_f64(O.unit_seed(seed0, 0, i, 0), (3 * i, 5 * i, 7 * i), *d, sigma=sigma)
            for i, d in enumerate(dims)]


def pack(wc, boxes, dtype=np.float64, offsets=None):
    dims = [(b.shape[2], b.shape[1], b.shape[0]) for b in boxes]
    units, n, extent = wc.capi.make_units(dims, offsets=offsets)
    cells = np.zeros(max(extent, 1), dtype)
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        cells[o:o + b.size] = b.ravel().astype(dtype)
    return units, n, extent, cells


def set_path(ctx, path):
    """Library options of a path ("staged" = the defaults)."""
    ctx.set_option(WC_OPT_SPARSE, 0 if path == "dense" else 1)
    ctx.set_option(WC_OPT_ORDERED, 0 if path == "tickets" else 1)
    ctx.set_option(WC_OPT_INVERSE_ROWS, 0 if path == "dense_inverse" else 1)


def gpu_payloads(wc, ctx, boxes, keep, dtype=np.float64, offsets=None, path="staged"):
    units, n, extent, cells = pack(wc, boxes, dtype, offsets)
    set_path(ctx, path)
    try:
        payload, offs, kept = ctx.forward_host(cells, units, n, keep)
    finally:
        set_path(ctx, "staged")  # library defaults
    return [wc.capi.unit_payload(payload, offs, kept, i) for i in range(n)], kept


def oracle_payload(O, b, keep):
    b32 = O.narrow(b) if b.dtype == np.float64 else b
    return O.compress_payload(b32, keep)[0]


# Forward paths, all byte-identical: the library default (sparse staging of
# 32-coefficient segments, look-back tile index from the launch order);
# "dense" staging (WC_OPT_SPARSE 0); "tickets": the look-back tile index from
# per-unit ticket atomics (WC_OPT_ORDERED 0: no dispatch-order assumption).
PATHS = ["staged", "dense", "tickets"]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("keep", KEEPS)
def test_forward_payload_bit_exact_fp64(wc, ctx, oracle, keep, path):
    boxes = synth(oracle, DIMS)
    got, kept = gpu_payloads(wc, ctx, boxes, keep, path=path)
    for i, b in enumerate(boxes):
        want = oracle_payload(oracle, b, keep)
        assert got[i] == want, f"unit {i} dims {DIMS[i]} keep {keep}"


@pytest.mark.parametrize("path", PATHS)
def test_forward_payload_bit_exact_fp32_input(wc, ctx, oracle, path):
    keep = KEEPS[1]
    boxes = [oracle.narrow(b) for b in synth(oracle, DIMS, seed0=1)]
    got, _ = gpu_payloads(wc, ctx, boxes, keep, dtype=np.float32, path=path)
    for i, b in enumerate(boxes):
        assert got[i] == oracle.compress_payload(b, keep)[0], f"unit {i} dims {DIMS[i]}"


@pytest.mark.parametrize("path", PATHS)
def test_unaligned_offsets(wc, ctx, oracle, path):
    """Odd cell offsets disable the vector loads; results must not change."""
    keep = KEEPS[1]
    dims = [(8, 8, 8), (6, 4, 2), (16, 2, 4), (4, 4, 16)]
    boxes = synth(oracle, dims, seed0=2)
    offs = [1, 1 + 512 + 3, 1 + 512 + 3 + 48 + 5, 1 + 512 + 3 + 48 + 5 + 128 + 7]
    got, _ = gpu_payloads(wc, ctx, boxes, keep, offsets=offs, path=path)
    for i, b in enumerate(boxes):
        assert got[i] == oracle_payload(oracle, b, keep)


def test_transform_bit_exact(wc, ctx, oracle):
    import torch
    boxes = [oracle.narrow(b) for b in synth(oracle, DIMS, seed0=3, sigma=3.0)]
    units, n, extent, cells = pack(wc, boxes, np.float32)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(cells).to(dev)
    d_flat = torch.full((max(extent, 1),), float("nan"), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    ctx.decompose(d_in.data_ptr(), wc.capi.WC_F32, units, n, d_flat.data_ptr())
    ctx.synchronize()
    flat = d_flat.cpu().numpy()
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        want = oracle.wavelet_decompose(b)
        assert flat[o:o + b.size].tobytes() == want.tobytes(), f"dims {DIMS[i]}"


def test_transform_extreme_values(wc, ctx, oracle):
    """Denormals, huge magnitudes (overflowing float adds), signed zeros."""
    import torch
    rng = np.random.default_rng(7)
    dims = [(8, 6, 4), (5, 3, 7)]
    boxes = []
    for (W, H, D) in dims:
        mant = rng.standard_normal((D, H, W))
        expo = rng.integers(-149, 128, (D, H, W))
        b = (mant * np.exp2(expo.astype(np.float64))).astype(np.float32)
        b[0, 0, :2] = [np.float32(1e-45), np.float32(-1e-45)]
        b[1, 0, :2] = [np.float32(3.4e38), np.float32(3.4e38)]
        b[0, 1, :2] = [np.float32(-0.0), np.float32(0.0)]
        boxes.append(b)
    units, n, extent, cells = pack(wc, boxes, np.float32)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(cells).to(dev)
    d_flat = torch.zeros(max(extent, 1), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    ctx.decompose(d_in.data_ptr(), wc.capi.WC_F32, units, n, d_flat.data_ptr())
    ctx.synchronize()
    flat = d_flat.cpu().numpy()
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        assert flat[o:o + b.size].tobytes() == oracle.wavelet_decompose(b).tobytes()


def special_boxes():
    out = {}
    b = np.full((4, 4, 4), 5.0, np.float32); b[1, 2, 3] = 7.5
    out["plus5_spike"] = (b, 15)
    out["minus5_sign_quirk"] = (np.full((4, 4, 4), -5.0, np.float32), 64)
    out["plus5"] = (np.full((4, 4, 4), 5.0, np.float32), 8)
    out["zeros"] = (np.zeros((4, 6, 8), np.float32), 0)
    b = np.zeros((4, 4, 4), np.float32); b[0, 0, 0] = 3.0; b[0, 0, 1] = -3.0
    out["tie_pm"] = (b, None)
    b = np.full((4, 4, 4), 2.0, np.float32); b[0, 0, 0] = np.nan; b[0, 0, 1] = np.nan
    b[0, 1, 0] = np.nan; b[0, 1, 1] = np.nan; b[1, 0, 0] = np.nan; b[1, 0, 1] = np.nan
    b[1, 1, 0] = np.nan; b[1, 1, 1] = np.nan
    out["nan_first"] = (b, 0)
    b = np.full((4, 4, 4), 2.0, np.float32); b[3, 3, 3] = np.nan
    out["nan_later"] = (b, None)
    b = np.full((2, 2, 4), 1.0, np.float32); b[0, 0, 0] = np.inf
    out["inf"] = (b, None)
    b = np.full((2, 4, 2), np.float32(1e-40), np.float32); b[1, 1, 1] = np.float32(3e-39)
    out["denormal"] = (b, None)
    out["const_3902"] = (np.full((64, 32, 16), np.float32(3902.4), np.float32), 4096)
    # the same quirks on fast-transform shapes (even W, H and D % 8 == 0)
    b = np.full((8, 4, 4), 5.0, np.float32); b[5, 2, 3] = 7.5
    out["plus5_spike_f"] = (b, 23)
    out["minus5_sign_quirk_f"] = (np.full((8, 4, 4), -5.0, np.float32), 128)
    out["zeros_f"] = (np.zeros((16, 6, 8), np.float32), 0)
    b = np.zeros((8, 4, 4), np.float32); b[3, 2, 2] = 3.0; b[3, 2, 3] = -3.0; b[7, 3, 1] = -3.0
    out["tie_pm_f"] = (b, None)
    b = np.full((8, 4, 4), 2.0, np.float32); b[:2, :2, :2] = np.nan
    out["nan_first_f"] = (b, 0)
    b = np.full((8, 4, 4), 2.0, np.float32); b[7, 3, 3] = np.nan
    out["nan_later_f"] = (b, None)
    b = np.full((8, 2, 2), 1.0, np.float32); b[4, 0, 0] = -np.inf
    out["inf_f"] = (b, None)
    b = np.full((8, 4, 2), np.float32(1e-40), np.float32); b[6, 1, 1] = np.float32(-3e-39)
    out["denormal_f"] = (b, None)
    b = np.full((16, 8, 8), 1.0, np.float32); b[9, 7, 6] = -50.0
    out["neg_max_f"] = (b, None)
    # negative signed max on sparse-staged shapes (D >= 32, hz % TZ == 0): thresh < 0
    # keeps every coefficient, including the segments the sparse staging skipped
    # (a lone negative spike: its block's 8 coefficients tie in |c|, the first in flat
    # order -- the negative low-pass one -- is the signed max)
    b = np.zeros((32, 16, 16), np.float32); b[9, 7, 6] = -50.0
    out["neg_max_sparse"] = (b, 32 * 16 * 16)
    rng = np.random.default_rng(5)
    b = (rng.standard_normal((64, 32, 32)) * 0.01).astype(np.float32)
    b[40:42, 2:4, 16:18] = 0.0; b[40, 3, 17] = -900.0
    out["neg_max_sparse_tiles"] = (b, 64 * 32 * 32)
    return out


@pytest.mark.parametrize("path", PATHS)
def test_special_boxes(wc, ctx, oracle, path):
    keep = KEEPS[1]
    sp = special_boxes()
    names = list(sp)
    got, kept = gpu_payloads(wc, ctx, [sp[k][0] for k in names], keep, dtype=np.float32, path=path)
    for i, k in enumerate(names):
        b, expect_kept = sp[k]
        want, wk = oracle.compress_payload(b, keep)
        assert got[i] == want, k
        if expect_kept is not None:
            assert wk == expect_kept == int(kept[i]), k


def test_empty_and_degenerate_units(wc, ctx, oracle):
    keep = KEEPS[1]
    boxes = [np.zeros((0, 3, 3), np.float32), np.ones((1, 1, 1), np.float32) * 4,
             np.zeros((3, 0, 2), np.float32), np.arange(6, dtype=np.float32).reshape(1, 1, 6)]
    got, kept = gpu_payloads(wc, ctx, boxes, keep, dtype=np.float32)
    for i, b in enumerate(boxes):
        if b.size == 0:
            D, H, W = b.shape
            assert got[i] == np.array([W, H, D, 0, 0], "<i4").tobytes()
        else:
            assert got[i] == oracle.compress_payload(b, keep)[0]


@pytest.mark.parametrize("path", ["staged", "tickets", "dense_inverse"])
@pytest.mark.parametrize("keep", [KEEPS[0], KEEPS[2]])
def test_inverse_bit_exact(wc, ctx, oracle, keep, path):
    boxes = synth(oracle, DIMS, seed0=4)
    units, n, extent, cells = pack(wc, boxes)
    payload, offs, kept = ctx.forward_host(cells, units, n, keep)
    set_path(ctx, path)
    try:
        regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
    finally:
        set_path(ctx, "staged")
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        p = wc.capi.unit_payload(payload, offs, kept, i)
        want = oracle.decompress_payload(p).ravel()
        assert regen[o:o + b.size].tobytes() == want.tobytes(), f"dims {DIMS[i]}"


@pytest.mark.parametrize("sparse", [1, 0])
def test_inverse_writes_every_coefficient(wc, ctx, oracle, sparse):
    """The decode writes zeros between pairs instead of clearing its scratch first: an
    inverse right after a dense one, over sparse, empty-payload (all-zero, NaN-first) and
    sign-quirk units, must equal the oracle's decompress exactly."""
    ctx.set_option(WC_OPT_SPARSE, sparse)
    dense = synth(oracle, [(32, 32, 32)] * 4 + [(64, 16, 8)], seed0=15)
    units, n, extent, cells = pack(wc, dense)
    payload, offs, kept = ctx.forward_host(cells, units, n, KEEPS[0])
    ctx.inverse_host(payload, offs[:n], units, n, extent)
    sp = special_boxes()
    boxes = [sp[k][0] for k in ("zeros_f", "nan_first_f", "plus5_spike_f", "const_3902", "minus5_sign_quirk_f",
                                "zeros", "tie_pm")]
    boxes.append(np.zeros((32, 32, 32), np.float32))
    boxes.append(oracle.narrow(synth(oracle, [(64, 64, 64)], seed0=16)[0]))
    units, n, extent, cells = pack(wc, boxes, np.float32)
    payload, offs, kept = ctx.forward_host(cells, units, n, KEEPS[2])
    regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
    ctx.set_option(WC_OPT_SPARSE, 1)
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        want = oracle.decompress_payload(wc.capi.unit_payload(payload, offs, kept, i)).ravel()
        assert regen[o:o + b.size].tobytes() == want.tobytes(), i


def test_inverse_repeated_calls_epoch_granules(wc, ctx, oracle):
    """The row index keeps its work items and look-back granules across calls,
    tagged with the call's epoch instead of zeroed: a big batch, then a smaller
    one (the big call's items past its end are stale), a malformed payload, the
    ticket form, and more than 256 units (the item workgroups' own look-back)
    must each decode exactly, on one context."""
    big_dims = [(64, 64, 64)] * 3 + [(32, 32, 32)] * 5 + [(16, 16, 16)] * 8
    small_dims = [(16, 16, 16), (8, 8, 8)]
    many_dims = [(8, 4, 8)] * 300 + [(32, 16, 64)] * 4
    batches = [(big_dims, 21), (small_dims, 22), (big_dims, 23), (many_dims, 24), (small_dims, 25)]

    def run(dims, seed, path="staged"):
        boxes = synth(oracle, dims, seed0=seed)
        units, n, extent, cells = pack(wc, boxes)
        payload, offs, kept = ctx.forward_host(cells, units, n, KEEPS[1])
        set_path(ctx, path)
        try:
            regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
        finally:
            set_path(ctx, "staged")
        for i, b in enumerate(boxes):
            o = units[i].cell_offset
            want = oracle.decompress_payload(wc.capi.unit_payload(payload, offs, kept, i)).ravel()
            assert regen[o:o + b.size].tobytes() == want.tobytes(), (dims[i], i, path)

    for dims, seed in batches:
        run(dims, seed)
    run(big_dims, 26, path="tickets")
    b = synth(oracle, [(8, 8, 8)], seed0=6)[0]
    p = bytearray(oracle_payload(oracle, b, KEEPS[1]))
    p[0] = 9
    units, n, extent = wc.capi.make_units([(8, 8, 8)])
    buf = np.zeros(len(p) + 16, np.uint8)
    buf[4:4 + len(p)] = np.frombuffer(bytes(p), np.uint8)
    with pytest.raises(wc.WaveletError):
        ctx.inverse_host(buf, np.array([4], np.uint64), units, n, extent)
    run(small_dims, 27)
    run(big_dims, 28)


def test_inverse_flat_random(wc, ctx, oracle):
    import torch
    rng = np.random.default_rng(11)
    dims = [(6, 10, 14), (3, 5, 7), (64, 8, 32), (2, 2, 2), (9, 9, 9)]
    flats = [(rng.standard_normal(W * H * D) * 100).astype(np.float32) for (W, H, D) in dims]
    units, n, extent = wc.capi.make_units(dims)
    f = np.zeros(extent, np.float32)
    for i, x in enumerate(flats):
        f[units[i].cell_offset:units[i].cell_offset + x.size] = x
    dev = torch.device("cuda", 0)
    d_f = torch.from_numpy(f).to(dev)
    d_o = torch.full((extent,), 123.0, dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    ctx.inverse_flat(d_f.data_ptr(), units, n, d_o.data_ptr())
    ctx.synchronize()
    out = d_o.cpu().numpy()
    for i, (W, H, D) in enumerate(dims):
        o = units[i].cell_offset
        want = oracle.inverse_wavelet_decompose(flats[i], W, H, D).ravel()
        assert out[o:o + W * H * D].tobytes() == want.tobytes(), dims[i]


def test_rmse(wc, ctx, oracle):
    import torch
    boxes = synth(oracle, DIMS[:12], seed0=5)
    keep = KEEPS[0]
    units, n, extent, cells = pack(wc, boxes)
    payload, offs, kept = ctx.forward_host(cells, units, n, keep)
    regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
    dev = torch.device("cuda", 0)
    d_a = torch.from_numpy(cells).to(dev)
    d_r = torch.from_numpy(regen).to(dev)
    d_out = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.rmse(d_a.data_ptr(), wc.capi.WC_F64, d_r.data_ptr(), units, n, d_out.data_ptr())
    ctx.synchronize()
    got = d_out.cpu().numpy()
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        want = oracle.rmse(oracle.narrow(b), regen[o:o + b.size].reshape(b.shape))
        assert got[i] == pytest.approx(want, rel=1e-12, abs=1e-300), DIMS[i]


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("shift", [(0, 0), (1, 0), (0, 1), (1, 1)])
def test_rmse_base_alignment(wc, ctx, oracle, dtype, shift):
    """wc_rmse (K7) with the originals and / or the reconstruction one element
    past a pair-aligned base: the pair-vector loads run only where both bases
    allow them, the scalar loop otherwise; every RMSE within 1e-12 of the oracle
    (odd-length units included: the vector path's tail cell)."""
    import torch
    dims = DIMS
    boxes = synth(oracle, dims, seed0=41)
    units, n, extent, cells = pack(wc, boxes, dtype)
    payload, offs, kept = ctx.forward_host(cells, units, n, KEEPS[1])
    regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
    dev = torch.device("cuda", 0)
    sa, sr = shift
    d_a = torch.from_numpy(np.concatenate([np.zeros(1, cells.dtype), cells])).to(dev)[1:] if sa \
        else torch.from_numpy(cells).to(dev)
    d_r = torch.from_numpy(np.concatenate([np.zeros(1, np.float32), regen])).to(dev)[1:] if sr \
        else torch.from_numpy(regen).to(dev)
    assert (d_a.data_ptr() % (2 * cells.itemsize) != 0) == bool(sa)
    assert (d_r.data_ptr() % 8 != 0) == bool(sr)
    d_out = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    code = wc.capi.WC_F64 if dtype == np.float64 else wc.capi.WC_F32
    ctx.rmse(d_a.data_ptr(), code, d_r.data_ptr(), units, n, d_out.data_ptr())
    ctx.synchronize()
    got = d_out.cpu().numpy()
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        orig = oracle.narrow(b) if dtype == np.float64 else b.astype(np.float32)
        want = oracle.rmse(orig, regen[o:o + b.size].reshape(b.shape))
        assert got[i] == pytest.approx(want, rel=1e-12, abs=1e-300), (dims[i], shift)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("which", ["rows", "mixed"])
def test_inverse_rmse_fused(wc, ctx, oracle, dtype, which):
    """wc_inverse_rmse: the reconstruction byte-equal to wc_inverse's and the
    per-box RMSE within 1e-12 of the oracle's calc_rmse_per_box on it.  "rows":
    every unit row-indexed (the fused pass); "mixed": odd dims put units on the
    dense decode, so the call runs wc_inverse + wc_rmse."""
    import torch
    dims = ([(64, 64, 64), (32, 16, 64), (16, 16, 16), (8, 4, 8), (2, 2, 2), (48, 32, 16), (66, 2, 130),
             (40, 40, 70), (32, 32, 32)] if which == "rows" else DIMS)
    boxes = synth(oracle, dims, seed0=31)
    units, n, extent, cells = pack(wc, boxes, dtype)
    payload, offs, kept = ctx.forward_host(cells, units, n, KEEPS[1])
    want_regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
    dev = torch.device("cuda", 0)
    d_p = torch.from_numpy(payload).to(dev)
    d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_a = torch.from_numpy(cells).to(dev)
    d_r = torch.full((extent,), float("nan"), dtype=torch.float32, device=dev)
    d_rm = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    code = wc.capi.WC_F64 if dtype == np.float64 else wc.capi.WC_F32
    torch.cuda.synchronize()
    for _ in range(2):  # part[] reused across calls
        ctx.inverse_rmse(d_p.data_ptr(), d_off.data_ptr(), units, n, d_a.data_ptr(), code, d_r.data_ptr(),
                         d_rm.data_ptr())
    ctx.synchronize()
    regen = d_r.cpu().numpy()
    got = d_rm.cpu().numpy()
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        assert regen[o:o + b.size].tobytes() == want_regen[o:o + b.size].tobytes(), dims[i]
        orig = oracle.narrow(b) if dtype == np.float64 else b.astype(np.float32)
        want = oracle.rmse(orig, regen[o:o + b.size].reshape(b.shape))
        assert got[i] == pytest.approx(want, rel=1e-12, abs=1e-300), dims[i]


def test_malformed_payload_rejected(wc, ctx, oracle):
    b = synth(oracle, [(8, 8, 8)], seed0=6)[0]
    p = bytearray(oracle_payload(oracle, b, KEEPS[1]))
    units, n, extent = wc.capi.make_units([(8, 8, 8)])
    offs = np.array([4], np.uint64)
    bad_dims = bytearray(p); bad_dims[0] = 9
    bad_run = bytearray(p); bad_run[20:24] = np.array([-5], "<i4").tobytes()
    for bad in (bad_dims, bad_run):
        buf = np.zeros(len(bad) + 16, np.uint8)
        buf[4:4 + len(bad)] = np.frombuffer(bytes(bad), np.uint8)
        with pytest.raises(wc.WaveletError) as ei:
            ctx.inverse_host(buf, offs, units, n, extent)
        assert ei.value.code == wc.capi.WC_ERR_FORMAT


@pytest.mark.parametrize("dims", [(4, 2, 2), (4, 2, 8)])  # generic (dense decode) and row-indexed shapes
@pytest.mark.parametrize("runs", [[0, 3, 10, 0], [0] * 40, [2] * 7 + [0] * 30, [15, 0, 0, 4], [0] * 64,
                                  [0] * 63 + [5], [70, 0], [], [63], [1] * 31 + [0] * 3])
def test_rle_decode_out_of_range_pairs_dropped(wc, ctx, oracle, runs, dims):
    """rle_decode drops pairs whose index reaches total (src/decompressor.cpp:20-27),
    also when the payload holds more pairs than coefficients (nrle > ncoeff); an
    empty payload and payloads that end exactly at ncoeff."""
    W, H, D = dims
    runs = np.array(runs, np.int32)
    vals = (np.arange(runs.size, dtype=np.float32) + 1.5).astype(np.float32)
    p = oracle.serialize(W, H, D, W * H * D, runs, vals)
    units, n, extent = wc.capi.make_units([(W, H, D)])
    buf = np.zeros(len(p) + 16, np.uint8)
    buf[4:4 + len(p)] = np.frombuffer(p, np.uint8)
    out = ctx.inverse_host(buf, np.array([4], np.uint64), units, n, extent)
    flat = oracle.rle_decode(runs, vals, W * H * D)
    want = oracle.inverse_wavelet_decompose(flat, W, H, D).ravel()
    assert out.tobytes() == want.tobytes()


def test_format_error_survives_later_calls(wc, ctx, oracle):
    """A malformed payload in an async wc_inverse is reported at the next
    synchronisation even when a forward (whose emit can raise errors too) runs in
    between; the error word is cleared once read."""
    import torch
    b = synth(oracle, [(8, 8, 8)], seed0=6)[0]
    p = bytearray(oracle_payload(oracle, b, KEEPS[1]))
    p[0] = 9  # W mismatch
    units, n, extent = wc.capi.make_units([(8, 8, 8)])
    dev = torch.device("cuda", 0)
    host = np.zeros(len(p) + 16, np.uint8)
    host[4:4 + len(p)] = np.frombuffer(bytes(p), np.uint8)
    d_pay = torch.from_numpy(host).to(dev)
    d_off = torch.tensor([4], dtype=torch.int64, device=dev)
    d_out = torch.zeros(extent, dtype=torch.float32, device=dev)
    cells = torch.from_numpy(b.ravel().copy()).to(dev)
    cap = wc.capi.payload_bound(units, n)
    d_p2 = torch.zeros(cap, dtype=torch.uint8, device=dev)
    d_o2 = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_k2 = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def fwd():
        ctx.forward(cells.data_ptr(), wc.capi.WC_F64, units, n, KEEPS[1], d_p2.data_ptr(), cap,
                    d_o2.data_ptr(), d_k2.data_ptr())

    ctx.inverse(d_pay.data_ptr(), d_off.data_ptr(), units, n, d_out.data_ptr())
    fwd()
    with pytest.raises(wc.WaveletError) as ei:
        ctx.synchronize()
    assert ei.value.code == wc.capi.WC_ERR_FORMAT
    fwd()
    ctx.synchronize()  # cleared once read: the next check is clean


@pytest.mark.parametrize("path", PATHS)
def test_large_batch_64cubed_fp64(wc, ctx, oracle, path):
    """64 boxes of the headline shape (64^3 fp64, keep 0.999f): every payload byte."""
    keep = KEEPS[1]
    dims = [(64, 64, 64)] * 64
    boxes = [oracle.synth_box_f64(oracle.unit_seed(0, 0, i, 0), (64 * (i % 8), 64 * (i // 8), 0), 64, 64, 64)
             for i in range(64)]
    got, kept = gpu_payloads(wc, ctx, boxes, keep, path=path)
    frac = kept.sum() / (64 * 64 ** 3)
    assert 0.05 < frac < 0.95
    for i, b in enumerate(boxes):
        assert got[i] == oracle_payload(oracle, b, keep), i


@pytest.mark.parametrize("path", PATHS)
def test_128cubed_fp32_and_mixed_sizes(wc, ctx, oracle, path):
    """C5 shape (128^3 fp32, keep 0.9999f: z split over tiles) beside fast-transform and
    other AMR-style mixed boxes in one batch."""
    keep = KEEPS[2]
    dims = [(128, 128, 128), (32, 32, 32), (16, 16, 16), (48, 32, 16), (64, 64, 64), (128, 64, 32)]
    boxes = [oracle.narrow(b) for b in synth(oracle, dims, seed0=8)]
    got, _ = gpu_payloads(wc, ctx, boxes, keep, dtype=np.float32, path=path)
    for i, b in enumerate(boxes):
        assert got[i] == oracle.compress_payload(b, keep)[0], dims[i]


def test_reference_wavelet_decomposition_case(wc):
    """Mirror of src/compressor.cpp:369-384: 4x8x16 box, round trip within 1e-6."""
    box = np.full((16, 8, 4), 5.0, np.float32)
    for (x, y, z, v) in [(1, 2, 3, 8.5), (2, 5, 6, 5.44), (1, 1, 1, 3.3999932),
                         (2, 2, 2, 3.19229), (3, 5, 12, 199.39029)]:
        box[z, y, x] = np.float32(v)
    flat = wc.wavelet_decompose(box)
    back = wc.inverse_wavelet_decompose(flat, 4, 8, 16)
    assert np.all(np.abs(back - box) <= 1e-6)


def test_reference_file_writing_case(wc, tmp_path):
    """Mirror of src/compressor.cpp:387-406: const 5.0 box, keep 0.999, exact through xz."""
    box = np.full((16, 8, 4), 5.0, np.float32)
    wc.compress([box], [0], 0.999, 0, 0, 0, str(tmp_path))
    back = wc.decompress(str(tmp_path / "compressed-wavelet-0-0-0-0.xz"), 0, 0, 0, 0)
    assert np.array_equal(back, box)


def test_python_mirror_compress_payloads(wc, oracle):
    """codec.compress_payloads (the Python mirror's batched compress(): each
    box uploaded from its own array, wc_forward_host_units) over mixed shapes
    and keeps: the oracle's bytes, and decompress_payloads inverts them."""
    boxes = [oracle.narrow(b) for b in synth(oracle, DIMS, seed0=29)]
    for keep in KEEPS:
        got = wc.compress_payloads(boxes, keep)
        for i, b in enumerate(boxes):
            assert got[i] == oracle.compress_payload(b, keep)[0], (keep, i)
        back = wc.decompress_payloads(got)
        for i, b in enumerate(boxes):
            if b.size:
                assert back[i].tobytes() == oracle.decompress_payload(got[i]).tobytes(), (keep, i)


def test_reference_calc_rmse_case(wc):
    """Mirror of src/calc-loss.cpp:68-86: {3.5, 3.5}."""
    a = [np.zeros((2, 2, 2), np.float32)] * 2
    p = [np.full((2, 2, 2), 3.5, np.float32)] * 2
    assert wc.calc_rmse_per_box(a, p, 2) == [3.5, 3.5]


@pytest.mark.parametrize("path", PATHS)
def test_gpu_matches_committed_golden_fixtures(wc, ctx, path):
    """Stored vectors (tests/golden/codec_golden.npz): payload bytes and reconstructions."""
    import json
    from pathlib import Path
    g = Path(__file__).parent / "golden"
    z = np.load(g / "codec_golden.npz")
    meta = json.loads((g / "codec_golden.json").read_text())
    by_keep = {}
    for case in meta["cases"]:
        by_keep.setdefault(case["keep"], []).append(case)
    for keep, cases in by_keep.items():
        boxes = [z[c["box"]] for c in cases]
        got, kept = gpu_payloads(wc, ctx, boxes, keep, dtype=np.float32, path=path)
        for i, c in enumerate(cases):
            assert got[i] == z[c["name"] + "/payload"].tobytes(), c["name"]
            assert int(kept[i]) == c["kept"], c["name"]
        regen = wc.decompress_payloads(got)
        for i, c in enumerate(cases):
            assert regen[i].tobytes() == z[c["name"] + "/regen"].tobytes(), c["name"]


SPARSE_DIMS = [(64, 64, 64), (16, 32, 64), (32, 8, 128), (64, 64, 64), (8, 2, 64), (64, 64, 64), (32, 32, 32),
               (16, 16, 32), (8, 8, 16), (2, 4, 96)]


@pytest.mark.parametrize("keep", [float(np.float32(k)) for k in (0.999, 0.5, 1.0, 1.5)])
def test_sparse_staging_sign_and_keep_edges(wc, ctx, oracle, keep):
    """Sparse staging (32-coefficient flat segments, D % 64 == 0 units) against
    the oracle where its tile bound matters: a unit whose signed max is NEGATIVE
    in one tile while the other tiles are positive (thresh < 0: every
    coefficient kept, re-staged densely), an all-negative field, keep = 1
    (thresh 0) and keep > 1 (thresh < 0 for positive maxima)."""
    boxes = synth(oracle, SPARSE_DIMS, seed0=9)
    boxes[1] = -boxes[1]                       # all-negative field
    boxes[3] = boxes[3].copy()
    boxes[3][40, 40, 40] = -1.0e6              # one negative spike: signed max < 0
    boxes[5] = boxes[5].copy()
    boxes[5][:, :, :] *= 1e-3
    boxes[5][3, 3, 3] = 2.0e4                  # one positive spike far above the rest
    for path in ("staged", "dense"):
        got, _ = gpu_payloads(wc, ctx, boxes, keep, path=path)
        for i, b in enumerate(boxes):
            assert got[i] == oracle_payload(oracle, b, keep), f"{path} unit {i} dims {SPARSE_DIMS[i]} keep {keep}"


@pytest.mark.parametrize("keep", [float(np.float32(k)) for k in (0.5, 0.99, 0.9999)])
def test_sparse_decode_tile_boundaries(wc, ctx, oracle, keep):
    """4096-pair decode tiles end mid-row; dense payloads (keep 0.5) put tile ends
    everywhere.  Reconstruction must equal the oracle's with WC_OPT_SPARSE on and
    off (payloads from the sparse-staged forward)."""
    boxes = synth(oracle, [(64, 64, 64), (32, 32, 32), (16, 16, 32), (64, 8, 64), (48, 32, 16)], seed0=21)
    units, n, extent, cells = pack(wc, boxes)
    payload, offs, kept = ctx.forward_host(cells, units, n, keep)
    for sparse in (1, 0):
        ctx.set_option(WC_OPT_SPARSE, sparse)
        regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
        for i, b in enumerate(boxes):
            o = units[i].cell_offset
            want = oracle.decompress_payload(wc.capi.unit_payload(payload, offs, kept, i)).ravel()
            assert regen[o:o + b.size].tobytes() == want.tobytes(), (sparse, i)
    ctx.set_option(WC_OPT_SPARSE, 1)


def test_sparse_staging_special_values(wc, ctx, oracle):
    """The reference's quirks on sparse-staged shapes (D = 32 and 64, 16/32-block z
    tiles): NaN first (nothing kept), NaN later, +inf, negative constant (sign
    quirk: everything kept -> dense re-staging), zeros, +M/-M ties, denormals."""
    def box(shape, fill, edits=()):
        b = np.full(shape, fill, np.float32)
        for idx, v in edits:
            b[idx] = v
        return b
    s1, s2, s3 = (32, 4, 4), (64, 4, 8), (64, 16, 64)
    boxes = [
        box(s1, 2.0, [((slice(0, 2), slice(0, 2), slice(0, 2)), np.nan)]),
        box(s1, 2.0, [((31, 3, 3), np.nan)]),
        box(s2, 1.0, [((0, 0, 0), np.inf)]),
        box(s2, 1.0, [((40, 2, 5), -np.inf)]),
        box(s1, -5.0),
        box(s2, 0.0),
        box(s2, 0.0, [((3, 2, 2), 3.0), ((3, 2, 3), -3.0), ((60, 3, 1), -3.0)]),
        box(s1, np.float32(1e-40), [((9, 1, 1), np.float32(3e-39))]),
        box(s2, 300.0, [((17, 1, 6), -1.0e5)]),
        # multi-tile units (8 z-tiles of 32 blocks): a negative field whose tiles all
        # stage densely, with all-NaN segments (stored too: thresh < 0 reads them
        # all); a positive field with one negative spike (mixed: re-staged)
        box(s3, -5.0, [((slice(None), slice(0, 2), slice(2, 4)), np.nan)]),
        box(s3, 7.0, [((slice(None), slice(0, 2), slice(2, 4)), np.nan), ((50, 12, 40), -2.0e4)]),
        box(s3, -7.0, [((20, 9, 33), 3.0e4)]),
    ]
    for keep in (KEEPS[1], 1.0):
        for path in ("staged", "dense"):
            got, _ = gpu_payloads(wc, ctx, boxes, keep, dtype=np.float32, path=path)
            for i, b in enumerate(boxes):
                assert got[i] == oracle.compress_payload(b, keep)[0], (path, keep, i)


def test_fallback_restage_past_one_round(wc, ctx, oracle):
    """k_transform_fallback checks units b, b + G, ... 256 at a time per
    workgroup (G = min(n, 2048)): with n > 2048 * 256 tiny two-tile units the
    needy ones (a positive tile staged sparsely, a negative spike in the other:
    thresh < 0, re-staged densely) sit in both check rounds; their payloads and
    a sample of the others equal the oracle's.  One host run (HOST_CHUNK 0)."""
    from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK
    n = 2048 * 256 + 777
    W, H, D = 2, 2, 128                      # nbz 64: two 32-block z tiles, sparse
    rng = np.random.default_rng(31)
    cells = (1.0 + 0.05 * rng.standard_normal((n, D, H, W))).astype(np.float32)
    needy = [3, 2047, 2048 * 255 + 5, 2048 * 256, 2048 * 256 + 1, n - 1]
    for u in needy:
        cells[u, 100:102] = -1.0e6           # a whole block in the second z tile: signed max < 0
    units, nu, extent = wc.capi.make_units([(W, H, D)] * n)
    assert nu == n and extent == cells.size  # 512-cell units pack back to back
    keep = KEEPS[1]
    ctx.set_option(WC_OPT_HOST_CHUNK, 0)
    try:
        payload, offs, kept = ctx.forward_host(cells.reshape(-1), units, n, keep)
    finally:
        ctx.set_option(WC_OPT_HOST_CHUNK, 1 << 25)
    for u in needy + [0, 1, 2048, 2048 * 256 - 1, 2048 * 256 + 2, n - 2]:
        want = oracle.compress_payload(cells[u], keep)[0]
        assert wc.capi.unit_payload(payload, offs, kept, u) == want, u
    for u in needy:
        assert int(kept[u]) == W * H * D, u  # thresh < 0: every coefficient kept


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_forward_host_pipelined_runs(wc, ctx, oracle, dtype):
    """wc_forward_host split into pipelined unit runs (WC_OPT_HOST_CHUNK small:
    many runs, cells uploaded run by run, payloads downloaded run by run)
    returns the same dense payload bytes, offsets and kept counts as one run,
    and every unit's payload equals the oracle's; also with gaps between the
    units' cells."""
    from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK
    keep = KEEPS[1]
    boxes = synth(oracle, DIMS, seed0=17)
    rng = np.random.default_rng(5)
    gaps = np.cumsum([0] + [int(b.size) + int(rng.integers(0, 9)) for b in boxes[:-1]]).tolist()
    for offsets in (None, gaps):
        units, n, extent, cells = pack(wc, boxes, dtype, offsets)
        ctx.set_option(WC_OPT_HOST_CHUNK, 0)
        p1, o1, k1 = ctx.forward_host(cells, units, n, keep)
        for chunk in (3000, 40000):
            ctx.set_option(WC_OPT_HOST_CHUNK, chunk)
            try:
                p2, o2, k2 = ctx.forward_host(cells, units, n, keep)
            finally:
                ctx.set_option(WC_OPT_HOST_CHUNK, 1 << 25)
            assert np.array_equal(o1, o2) and np.array_equal(k1[:n], k2[:n]), chunk
            for i in range(n):
                assert wc.capi.unit_payload(p2, o2, k2, i) == wc.capi.unit_payload(p1, o1, k1, i), (chunk, i)
        for i, b in enumerate(boxes):
            assert wc.capi.unit_payload(p1, o1, k1, i) == oracle_payload(oracle, b.astype(dtype), keep), i


def test_inverse_host_pipelined_runs(wc, ctx, oracle):
    """wc_inverse_host split into pipelined unit runs (payload spans uploaded
    run by run, boxes downloaded run by run in back-to-back spans) reconstructs
    the same values as one run, equal to the oracle's, also with gaps between
    the units' cells (the gap cells of the caller's buffer stay untouched) and
    with the units' payloads in reverse order."""
    from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK
    keep = KEEPS[1]
    boxes = synth(oracle, DIMS, seed0=23)
    rng = np.random.default_rng(6)
    gaps = np.cumsum([0] + [int(b.size) + int(rng.integers(0, 9)) for b in boxes[:-1]]).tolist()
    for offsets in (None, gaps):
        units, n, extent, cells = pack(wc, boxes, np.float64, offsets)
        payload, offs, kept = ctx.forward_host(cells, units, n, keep)
        # the same payloads laid out in reverse unit order
        blobs = [wc.capi.unit_payload(payload, offs, kept, i) for i in range(n)]
        rev = bytearray(4)
        roffs = np.zeros(n + 1, np.uint64)
        for i in reversed(range(n)):
            roffs[i] = len(rev)
            rev += blobs[i] + b"\0" * ((-len(blobs[i])) % 4)
        rev = np.frombuffer(bytes(rev), np.uint8)
        want = [oracle.decompress_payload(blobs[i]).ravel() for i in range(n)]
        for pay, po in ((payload, offs), (rev, roffs)):
            for chunk in (0, 3000, 40000):
                ctx.set_option(WC_OPT_HOST_CHUNK, chunk)
                try:
                    regen = ctx.inverse_host(pay, po[:n], units, n, extent)
                finally:
                    ctx.set_option(WC_OPT_HOST_CHUNK, 1 << 25)
                owned = np.zeros(extent, bool)
                for i, b in enumerate(boxes):
                    o = units[i].cell_offset
                    owned[o:o + b.size] = True
                    assert regen[o:o + b.size].tobytes() == want[i].tobytes(), (chunk, i)
                assert not regen[~owned].any(), chunk  # gap cells untouched


@pytest.mark.parametrize("threads,thp", [(0, 1), (1, 0), (4, 1), (-1, 1), (-1, 0)])
def test_host_destination_prefault(wc, ctx, oracle, threads, thp):
    """WC_OPT_HOST_THREADS / WC_OPT_HOST_THP: the _host calls fault in each
    destination span of the caller's buffer just before its device-to-host
    copy (csrc/wc_hostmem.h).  Into caller buffers that already hold data,
    over pipelined runs: the payload bytes before 4 and past offsets[n] and
    the output's gap cells (whole pages of sentinels between the units) keep
    their values, and every setting gives the same bytes as the oracle."""
    from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK, WC_OPT_HOST_THP, WC_OPT_HOST_THREADS
    keep = KEEPS[1]
    boxes = synth(oracle, [(64, 64, 64), (32, 64, 128), (64, 64, 64), (16, 16, 16), (64, 32, 64)], seed0=41)
    boxes = [b.astype(np.float32) for b in boxes]
    gap = 3 * 4096 + 5  # cells: more than two whole pages between units
    offsets = np.cumsum([0] + [int(b.size) + gap for b in boxes[:-1]]).tolist()
    units, n, extent, cells = pack(wc, boxes, np.float32, offsets)
    cap = wc.capi.payload_bound(units, n)
    payload = np.full(cap, 0xAB, np.uint8)
    offs = np.zeros(n + 1, np.uint64)
    kept = np.zeros(n, np.uint32)
    out = np.full(extent, 7.0, np.float32)
    ctx.set_option(WC_OPT_HOST_THREADS, threads)
    ctx.set_option(WC_OPT_HOST_THP, thp)
    ctx.set_option(WC_OPT_HOST_CHUNK, 1 << 18)
    try:
        ctx._check(ctx._L.wc_forward_host(ctx._h, cells.ctypes.data, wc.capi.WC_F32, units, n, float(keep),
                                          payload.ctypes.data, cap, offs.ctypes.data, kept.ctypes.data))
        ctx._check(ctx._L.wc_inverse_host(ctx._h, payload.ctypes.data, offs.ctypes.data, units, n,
                                          out.ctypes.data))
    finally:
        ctx.set_option(WC_OPT_HOST_THREADS, -1)
        ctx.set_option(WC_OPT_HOST_THP, 1)
        ctx.set_option(WC_OPT_HOST_CHUNK, 1 << 25)
    end = int(offs[n])
    assert np.all(payload[:4] == 0xAB) and np.all(payload[end + 4:] == 0xAB)
    owned = np.zeros(extent, bool)
    for i, b in enumerate(boxes):
        want = oracle_payload(oracle, b, keep)
        assert wc.capi.unit_payload(payload, offs, kept, i) == want, i
        o = units[i].cell_offset
        owned[o:o + b.size] = True
        assert out[o:o + b.size].tobytes() == oracle.decompress_payload(want).ravel().tobytes(), i
    assert np.all(out[~owned] == 7.0)


@pytest.mark.parametrize("chunk", [0, 1 << 21])
def test_host_uploads_from_pageable_memory(wc, ctx, oracle, chunk):
    """Large pageable sources (the cells of wc_forward_host, the payloads of
    wc_inverse_host: >= 64 MB here) go through the context's pinned bounce
    slots, copied by a host pool while earlier slots' DMA runs, also across
    pipelined unit runs (HOST_CHUNK 2^21: slots rotating across runs); the
    bytes equal the direct path's (WC_OPT_HOST_THREADS 0) and the oracle's."""
    from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK, WC_OPT_HOST_THREADS
    keep = float(np.float32(0.99999))  # most coefficients kept: a payload of ~80 MB
    boxes = synth(oracle, [(64, 64, 64)] * 40, seed0=71)
    units, n, extent, cells = pack(wc, boxes)
    assert cells.nbytes >= (64 << 20)
    ctx.set_option(WC_OPT_HOST_CHUNK, chunk)
    try:
        ctx.set_option(WC_OPT_HOST_THREADS, 0)
        p0, o0, k0 = ctx.forward_host(cells, units, n, keep)
        r0 = ctx.inverse_host(p0, o0[:n], units, n, extent)
        ctx.set_option(WC_OPT_HOST_THREADS, -1)
        p1, o1, k1 = ctx.forward_host(cells, units, n, keep)
        assert int(o1[n]) >= (64 << 20)
        r1 = ctx.inverse_host(p1, o1[:n], units, n, extent)
        r2 = ctx.inverse_host(p1.copy(), o1[:n], units, n, extent)  # a source the runtime has never seen
    finally:
        ctx.set_option(WC_OPT_HOST_THREADS, -1)
        ctx.set_option(WC_OPT_HOST_CHUNK, 1 << 25)
    end = int(o0[n])
    assert np.array_equal(o0, o1) and np.array_equal(k0, k1) and np.array_equal(p0[:end + 4], p1[:end + 4])
    assert np.array_equal(r0, r1) and np.array_equal(r0, r2)
    for i in (0, n - 1):
        want = oracle_payload(oracle, boxes[i], keep)
        assert wc.capi.unit_payload(p1, o1, k1, i) == want, i
        o = units[i].cell_offset
        assert r1[o:o + boxes[i].size].tobytes() == oracle.decompress_payload(want).ravel().tobytes(), i


def test_plan_cache_eviction(wc, ctx, oracle):
    """More distinct batches than the plan cache holds (16), each twice: plans
    are swapped back in, evicted, and rebuilt into an evicted plan's buffers;
    every payload still equals the oracle's, forward and inverse."""
    keep = KEEPS[1]
    batches = []
    for j in range(20):
        dims = [DIMS[(j + k) % len(DIMS)] for k in range(3)]
        batches.append(synth(oracle, dims, seed0=100 + j))
    for rep in range(2):
        for j, boxes in enumerate(batches):
            units, n, extent, cells = pack(wc, boxes)
            payload, offs, kept = ctx.forward_host(cells, units, n, keep)
            regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
            for i, b in enumerate(boxes):
                want = oracle_payload(oracle, b, keep)
                assert wc.capi.unit_payload(payload, offs, kept, i) == want, (rep, j, i)
                o = units[i].cell_offset
                assert regen[o:o + b.size].tobytes() == oracle.decompress_payload(want).ravel().tobytes(), (rep, j, i)


def test_two_contexts_on_one_device(wc, ctx, oracle):
    """A second live context on the same device (both in the launch-order
    form of the look-backs, which depends on no dispatch order); payloads and
    reconstructions stay the oracle's through the host-buffer calls."""
    keep = KEEPS[1]
    boxes = synth(oracle, DIMS, seed0=23)
    units, n, extent, cells = pack(wc, boxes)
    other = wc.capi.Context(0)
    try:
        for c in (ctx, other, ctx):
            payload, offs, kept = c.forward_host(cells, units, n, keep)
            regen = c.inverse_host(payload, offs[:n], units, n, extent)
            for i, b in enumerate(boxes):
                want = oracle_payload(oracle, b, keep)
                assert wc.capi.unit_payload(payload, offs, kept, i) == want, i
                o = units[i].cell_offset
                assert regen[o:o + b.size].tobytes() == oracle.decompress_payload(want).ravel().tobytes(), i
    finally:
        other.close()


def test_forward_host_runs_with_empty_units(wc, ctx, oracle):
    """Pipelined host runs (WC_OPT_HOST_CHUNK small) over a batch with empty
    units at its start, between boxes and at its end: the same bytes and
    offsets as one run; empty units serialize as a bare header."""
    from wavelet_compression_amd.capi import WC_OPT_HOST_CHUNK
    keep = KEEPS[1]
    real = synth(oracle, DIMS[:12], seed0=31)
    empty = np.zeros((0, 4, 4), np.float64)
    boxes = [empty] + [x for b in real for x in (b, empty)] + [empty, empty]
    units, n, extent, cells = pack(wc, boxes)
    ctx.set_option(WC_OPT_HOST_CHUNK, 0)
    p1, o1, k1 = ctx.forward_host(cells, units, n, keep)
    ctx.set_option(WC_OPT_HOST_CHUNK, 2000)
    try:
        p2, o2, k2 = ctx.forward_host(cells, units, n, keep)
    finally:
        ctx.set_option(WC_OPT_HOST_CHUNK, 1 << 25)
    assert np.array_equal(o1, o2) and np.array_equal(k1[:n], k2[:n])
    for i, b in enumerate(boxes):
        got = wc.capi.unit_payload(p2, o2, k2, i)
        assert got == wc.capi.unit_payload(p1, o1, k1, i), i
        if b.size == 0:
            D, H, W = b.shape
            assert got == np.array([W, H, D, 0, 0], "<i4").tobytes(), i
        else:
            assert got == oracle_payload(oracle, b, keep), i


@pytest.mark.parametrize("groups", [1, 2, 3, 7])
def test_inverse_unit_groups_pipelined(wc, ctx, oracle, groups):
    """The row-indexed inverse in unit groups (WC_OPT_INV_GROUPS: row index of
    group g + 1 beside K6r of group g on a second stream) reconstructs the
    oracle's cells for a batch mixing row-indexed and dense-decode units, alone
    and fused with the per-box RMSE; a batch of empty units gets RMSE 0."""
    import torch
    from wavelet_compression_amd.capi import WC_OPT_INV_GROUPS
    keep = KEEPS[1]
    dims = [(64, 64, 64), (16, 16, 16), (3, 5, 7), (32, 32, 32), (48, 32, 16), (6, 10, 14), (64, 8, 64),
            (2, 2, 8), (16, 32, 64), (32, 32, 32)]
    boxes = synth(oracle, dims, seed0=61)
    units, n, extent, cells = pack(wc, boxes)
    payload, offs, kept = ctx.forward_host(cells, units, n, keep)
    want = [oracle.decompress_payload(wc.capi.unit_payload(payload, offs, kept, i)).ravel() for i in range(n)]
    before = ctx.get_option(WC_OPT_INV_GROUPS)  # the session-scoped context keeps the library default afterwards
    ctx.set_option(WC_OPT_INV_GROUPS, groups)
    try:
        regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
        for i, b in enumerate(boxes):
            o = units[i].cell_offset
            assert regen[o:o + b.size].tobytes() == want[i].tobytes(), (groups, i)
        # fused inverse + RMSE over the row-indexed units only (device pointers)
        rix = [i for i, d in enumerate(dims) if d[0] % 2 == 0 and d[1] % 2 == 0 and d[2] % 8 == 0]
        rb = [boxes[i] for i in rix]
        ru, rn, rext, rcells = pack(wc, rb)
        rp, ro, rk = ctx.forward_host(rcells, ru, rn, keep)
        dev = torch.device("cuda", 0)
        d_p = torch.from_numpy(rp.copy()).to(dev)
        d_o = torch.from_numpy(ro[:rn].astype(np.int64)).to(dev)
        d_c = torch.from_numpy(rcells).to(dev)
        d_out = torch.zeros(rext, dtype=torch.float32, device=dev)
        d_r = torch.zeros(rn, dtype=torch.float64, device=dev)
        torch.cuda.synchronize()
        ctx.inverse_rmse(d_p.data_ptr(), d_o.data_ptr(), ru, rn, d_c.data_ptr(), wc.capi.WC_F64, d_out.data_ptr(),
                         d_r.data_ptr())
        ctx.synchronize()
        out, r = d_out.cpu().numpy(), d_r.cpu().numpy()
        for j, b in enumerate(rb):
            o = ru[j].cell_offset
            back = oracle.decompress_payload(wc.capi.unit_payload(rp, ro, rk, j))
            assert out[o:o + b.size].tobytes() == back.ravel().tobytes(), (groups, j)
            assert r[j] == pytest.approx(oracle.rmse(oracle.narrow(b), back), rel=1e-12, abs=1e-300), (groups, j)
        # every unit empty: the fused call still writes RMSE 0
        eu, en, _ = wc.capi.make_units([(0, 4, 8), (4, 0, 8)])
        d_r2 = torch.full((en,), 7.0, dtype=torch.float64, device=dev)
        ctx.inverse_rmse(d_p.data_ptr(), d_o.data_ptr(), eu, en, d_c.data_ptr(), wc.capi.WC_F64, d_out.data_ptr(),
                         d_r2.data_ptr())
        ctx.synchronize()
        assert d_r2.cpu().tolist() == [0.0, 0.0]
    finally:
        ctx.set_option(WC_OPT_INV_GROUPS, before)


def test_s32_shape_special_values(wc, ctx, oracle):
    """The specialised 32 x 1 x 32 transform tiles (wc_xform.h s32_ok: every C2 and
    C5 unit) take the max key only where |c| equals the tile's largest |c|, and
    test candidates in fp32 against the bound rounded toward -inf: the
    reference's quirks on that shape (64 x 16 x 64 and 64^3 boxes, cells at
    even offsets, fp32 and fp64) — NaN at flat index 0 (nothing kept), a NaN
    later, +/-inf, ties of +M and -M in different tiles (the first in flat order
    decides the sign: a negative max keeps everything, re-staged densely),
    -0.0 among zeros, constant fields (every coefficient ties), denormals — at
    keep 0.5, 0.999f, 1.0 and 1.5 (thresh < 0)."""
    def box(shape, fill, edits=()):
        b = np.full(shape, fill, np.float32)
        for idx, v in edits:
            b[idx] = v
        return b
    s, c = (64, 16, 64), (64, 64, 64)  # (D, H, W)
    rng = np.random.default_rng(32)
    noise = (rng.standard_normal(c) * 0.05 + 300.0).astype(np.float32)
    boxes = [
        box(s, 2.0, [((0, 0, 0), np.nan)]),                       # flat[0] NaN
        box(s, 2.0, [((40, 9, 33), np.nan)]),                     # a later NaN never wins
        box(s, 1.0, [((5, 3, 7), np.inf)]),
        box(s, 1.0, [((50, 12, 60), -np.inf)]),
        box(s, 0.0, [((9, 2, 40), 8.0), ((9, 2, 41), -8.0)]),     # +M / -M in one block
        box(s, 0.0, [((3, 1, 2), -8.0), ((60, 14, 62), 8.0)]),    # first (negative) spike wins
        box(s, 0.0, [((60, 14, 62), -8.0), ((3, 1, 2), 8.0)]),    # first (positive) spike wins
        box(s, 0.0, [((7, 5, 9), np.float32(-0.0)), ((8, 5, 9), np.float32(-0.0))]),
        box(s, 3.0),                                              # every LLL coefficient ties
        box(s, np.float32(1e-40), [((30, 8, 30), np.float32(3e-39))]),
        noise,
        -noise,
    ]
    for keep in (0.5, KEEPS[1], 1.0, 1.5):
        for dtype in (np.float32, np.float64):
            got, kept = gpu_payloads(wc, ctx, [b.astype(dtype) for b in boxes], keep, dtype=dtype)
            for i, b in enumerate(boxes):
                want, wk = oracle.compress_payload(b, keep)
                assert got[i] == want, (keep, dtype.__name__, i)
                assert int(kept[i]) == wk


def test_32xHx32_shape_special_values(wc, ctx, oracle):
    """The 16 x 4 x 16-block transform tiles of 32 x H x 32 boxes (H % 8 == 0: the
    32^3 units of C3 / C4; 16-coefficient sparse segments; a specialised body for
    them was measured and not kept, profiles/r06/experiments/gpu_s16.txt) on the
    same quirks as the S32 test above: NaN at flat index 0 and later, +/-inf,
    +M / -M ties in one block and across tiles, -0.0, constant fields, denormals,
    smooth noise of either sign — fp32 and fp64, keep 0.5, 0.999f, 1.0, 1.5."""
    def box(shape, fill, edits=()):
        b = np.full(shape, fill, np.float32)
        for idx, v in edits:
            b[idx] = v
        return b
    s, c, t = (32, 8, 32), (32, 32, 32), (32, 24, 32)  # (D, H, W)
    rng = np.random.default_rng(16)
    noise = (rng.standard_normal(c) * 0.05 + 300.0).astype(np.float32)
    boxes = [
        box(s, 2.0, [((0, 0, 0), np.nan)]),
        box(c, 2.0, [((20, 29, 17), np.nan)]),
        box(s, 1.0, [((5, 3, 7), np.inf)]),
        box(t, 1.0, [((30, 21, 30), -np.inf)]),
        box(c, 0.0, [((9, 2, 20), 8.0), ((9, 2, 21), -8.0)]),
        box(c, 0.0, [((3, 1, 2), -8.0), ((30, 30, 31), 8.0)]),
        box(c, 0.0, [((30, 30, 31), -8.0), ((3, 1, 2), 8.0)]),
        box(s, 0.0, [((7, 5, 9), np.float32(-0.0)), ((8, 5, 9), np.float32(-0.0))]),
        box(t, 3.0),
        box(c, np.float32(1e-40), [((30, 8, 30), np.float32(3e-39))]),
        noise,
        -noise,
        noise[:, :8, :] * np.float32(0.5),
    ]
    for keep in (0.5, KEEPS[1], 1.0, 1.5):
        for dtype in (np.float32, np.float64):
            got, kept = gpu_payloads(wc, ctx, [b.astype(dtype) for b in boxes], keep, dtype=dtype)
            for i, b in enumerate(boxes):
                want, wk = oracle.compress_payload(b, keep)
                assert got[i] == want, (keep, dtype.__name__, i)
                assert int(kept[i]) == wk


@pytest.mark.parametrize("seed", [101, 202])
def test_random_shapes_round_trip(wc, ctx, oracle, seed):
    """Seeded random batches over every tile class the planner picks (odd and even
    dims, D % 8 == 0 or not, sparse 16/32-coefficient segments, the specialised
    32 x 1 x 32 shape, row-indexed and dense-decode inverse units, unaligned cell
    offsets), random keep per batch and fp32/fp64 cells: payload bytes equal the
    oracle's (the reference's compress() without xz) and the reconstruction
    equals its decompress() bit for bit."""
    rng = np.random.default_rng(seed)
    sizes = [1, 2, 3, 5, 8, 16, 24, 32, 33, 48, 64, 66, 96, 128]
    dims = [tuple(int(rng.choice(sizes)) for _ in range(3)) for _ in range(36)]
    dims = [d for d in dims if d[0] * d[1] * d[2] <= 1 << 20][:28] + [(64, 64, 64), (128, 16, 64), (64, 32, 64)]
    boxes = synth(oracle, dims, seed0=seed, sigma=float(rng.choice([0.01, 0.05, 5.0])))
    keep = float(np.float32(rng.choice([0.5, 0.9, 0.99, 0.999, 0.9999, 1.0])))
    offsets = None
    if seed % 2:  # odd cell offsets: the unaligned-load and generic paths
        offsets, o = [], 1
        for d in dims:
            offsets.append(o)
            o += d[0] * d[1] * d[2] + 3
    for dtype in (np.float32, np.float64):
        units, n, extent, cells = pack(wc, boxes, dtype, offsets)
        payload, offs, kept = ctx.forward_host(cells, units, n, keep)
        regen = ctx.inverse_host(payload, offs[:n], units, n, extent)
        for i, b in enumerate(boxes):
            p = wc.capi.unit_payload(payload, offs, kept, i)
            assert p == oracle_payload(oracle, b.astype(dtype), keep), (dtype.__name__, dims[i], keep)
            o = units[i].cell_offset
            want = oracle.decompress_payload(p).ravel()
            assert regen[o:o + b.size].tobytes() == want.tobytes(), (dtype.__name__, dims[i], keep)
