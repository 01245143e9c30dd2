"""The cohort forward (wc_cohort.hip, WC_OPT_COHORT): K1 and the emit of large
S32-shape units in one persistent launch, staging through a ring that stays in
the Infinity Cache.  Its payloads must equal the staged two-kernel path's and
the CPU oracle's (the reference's compress() without xz, src/compressor.cpp:
192-248) byte for byte, for every cohort size / lag (ring reuse, a last
cohort shorter than the others), fp32 and fp64 cells, and the reference's
quirks (NaN first, a negative signed max keeping everything, all zeros, inf,
constant fields); a forced wait timeout surfaces as WC_ERR_HIP and the next
call is exact again."""
import numpy as np
import pytest
from wavelet_compression_amd.capi import WC_OPT_COHORT, WC_OPT_COHORT_LAG, WC_OPT_SPIN_LIMIT

pytestmark = pytest.mark.gpu

KEEPS = [float(np.float32(0.999)), float(np.float32(0.9999))]
# every shape has 32 x 1 x 32-block transform tiles, hx and hz multiples of 32, >= 2^21 cells
SHAPES = [(128, 128, 128), (64, 64, 512), (256, 64, 128), (64, 256, 128), (128, 256, 64)]


def _boxes(oracle, n, seed0):
    return [oracle.synth_box_f64(oracle.unit_seed(seed0, 1, i, 2), (16 * i, 8 * i, 4 * i), *SHAPES[i % len(SHAPES)])
            for i in range(n)]


def _pack(wc, boxes, dtype):
    dims = [(b.shape[2], b.shape[1], b.shape[0]) for b in boxes]
    units, n, extent = wc.capi.make_units(dims)
    cells = np.zeros(extent, dtype)
    for i, b in enumerate(boxes):
        o = units[i].cell_offset
        cells[o:o + b.size] = b.ravel().astype(dtype)
    return units, n, cells


def _run(wc, ctx, units, n, cells, keep, cohort, lag=2):
    ctx.set_option(WC_OPT_COHORT, cohort)
    ctx.set_option(WC_OPT_COHORT_LAG, lag)
    try:
        ctx.profile_enable(True)
        ctx.profile_read()
        payload, offs, kept = ctx.forward_host(cells, units, n, keep)
        stages = ctx.profile_read()
    finally:
        ctx.profile_enable(False)
        ctx.set_option(WC_OPT_COHORT, 0)
        ctx.set_option(WC_OPT_COHORT_LAG, 2)
    return [wc.capi.unit_payload(payload, offs, kept, i) for i in range(n)], stages


@pytest.fixture(scope="module")
def batch(wc, oracle):
    boxes = _boxes(oracle, 11, 5)
    return boxes, {dt: _pack(wc, boxes, dt) for dt in (np.float32, np.float64)}


@pytest.mark.parametrize("cohort,lag", [(1, 1), (2, 2), (3, 1), (4, 2), (16, 2)])
@pytest.mark.parametrize("keep", KEEPS)
def test_cohort_payloads_equal_staged_path(wc, ctx, oracle, batch, cohort, lag, keep):
    boxes, packed = batch
    for dt in (np.float32, np.float64):
        units, n, cells = packed[dt]
        want, st0 = _run(wc, ctx, units, n, cells, keep, 0)
        got, st1 = _run(wc, ctx, units, n, cells, keep, cohort, lag)
        assert "cohort" in st1 and "cohort" not in st0 and "emit" not in st1, (st0, st1)
        for i in range(n):
            assert got[i] == want[i], (dt, cohort, lag, i)
        for i in (0, n - 1):  # the oracle on the first and the last unit (last cohort, reused ring slot)
            b = oracle.narrow(boxes[i]) if dt == np.float64 else boxes[i].astype(np.float32)
            assert got[i] == oracle.compress_payload(b, keep)[0], (dt, i)


def test_cohort_special_values(wc, ctx, oracle):
    """The reference's quirks on the cohort path, one unit each: NaN at flat
    index 0 (thresh NaN: nothing kept), a NaN later, a negative signed max
    (thresh < 0: everything kept, no re-staging needed with dense staging), all
    zeros, +/-inf, a constant field (every coefficient ties), denormals."""
    keep = KEEPS[0]
    base = _boxes(oracle, 8, 17)
    b = [x.copy() for x in base]
    b[0][0, 0, 0] = np.nan
    b[0][0, 0, 1] = np.nan
    b[1][5, 7, 9] = np.nan
    b[2] = -(np.abs(b[2]) + 1.0)  # every cell negative: the largest |c| (the low-pass sub-band) is negative
    b[3][:] = 0.0
    b[4][3, 3, 3] = np.inf
    b[4][9, 9, 9] = -np.inf
    b[5][:] = 3.25
    b[6] *= 1e-41
    for dt in (np.float32, np.float64):
        units, n, cells = _pack(wc, b, dt)
        got, st = _run(wc, ctx, units, n, cells, keep, 2, 1)
        assert "cohort" in st
        for i in range(n):
            x = oracle.narrow(b[i]) if dt == np.float64 else b[i].astype(np.float32)
            want, k = oracle.compress_payload(x, keep)
            assert got[i] == want, (dt, i)
        hdr = np.frombuffer(got[2][:20], "<i4")
        assert hdr[4] == hdr[3]  # negative max: every coefficient kept


def test_cohort_not_taken_for_ineligible_batches(wc, ctx, oracle):
    """A batch with one small unit keeps the two-kernel path (same bytes)."""
    boxes = _boxes(oracle, 3, 23) + [oracle.synth_box_f64(7, (0, 0, 0), 64, 64, 64)]
    units, n, cells = _pack(wc, boxes, np.float32)
    got, st = _run(wc, ctx, units, n, cells, KEEPS[0], 4)
    assert "cohort" not in st and "emit" in st
    for i in range(n):
        assert got[i] == oracle.compress_payload(boxes[i].astype(np.float32), KEEPS[0])[0], i


def test_cohort_not_taken_in_ticket_form(wc, ctx, oracle, batch):
    """The cohort launch relies on in-order dispatch (one block per item); the
    ticket form (WC_OPT_ORDERED 0, shared devices) runs the two-kernel path."""
    from wavelet_compression_amd.capi import WC_OPT_ORDERED
    boxes, packed = batch
    units, n, cells = packed[np.float32]
    ctx.set_option(WC_OPT_ORDERED, 0)
    try:
        got, st = _run(wc, ctx, units, n, cells, KEEPS[1], 4, 1)
    finally:
        ctx.set_option(WC_OPT_ORDERED, 1)
    assert "cohort" not in st and "emit" in st
    assert got[3] == oracle.compress_payload(boxes[3].astype(np.float32), KEEPS[1])[0]


def test_cohort_wait_timeout_reported_then_exact(wc, ctx, oracle):
    """WC_OPT_SPIN_LIMIT 1: the first unanswered poll of a cohort wait fails;
    the call reports WC_ERR_HIP (no hang, no out-of-range access), and the
    next call with the default bound is exact.  On the session context (the
    only live one: a second context would take the ticket form, not the
    cohort); the timeout makes the ticket form sticky, reset afterwards."""
    import torch
    from wavelet_compression_amd.capi import WC_OPT_TICKETS
    boxes = _boxes(oracle, 6, 29)
    units, n, host = _pack(wc, boxes, np.float32)
    dev = torch.device("cuda", 0)
    cells = torch.from_numpy(host).to(dev)
    cap = wc.capi.payload_bound(units, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the fills above run on torch's stream, the context on its own
    c = ctx
    try:
        c.set_option(WC_OPT_COHORT, 1)
        c.set_option(WC_OPT_COHORT_LAG, 1)
        c.set_option(WC_OPT_SPIN_LIMIT, 1)
        c.profile_enable(True)
        c.profile_read()
        seen = False
        for _ in range(4):
            c.forward(cells.data_ptr(), wc.capi.WC_F32, units, n, KEEPS[0], payload.data_ptr(), cap,
                      offsets.data_ptr(), kept.data_ptr())
            try:
                c.synchronize()
            except wc.WaveletError as e:
                assert e.code == wc.capi.WC_ERR_HIP and "timed out" in str(e), e
                seen = True
                break
        assert "cohort" in c.profile_read()
        c.set_option(WC_OPT_SPIN_LIMIT, 0)
        c.set_option(WC_OPT_TICKETS, 0)
        c.forward(cells.data_ptr(), wc.capi.WC_F32, units, n, KEEPS[0], payload.data_ptr(), cap,
                  offsets.data_ptr(), kept.data_ptr())
        c.synchronize()
        assert "cohort" in c.profile_read()
        p, o, k = payload.cpu().numpy(), offsets.cpu().numpy(), kept.cpu().numpy()
        for i in range(n):
            got = p[int(o[i]):int(o[i]) + 20 + 8 * int(k[i])].tobytes()
            assert got == oracle.compress_payload(boxes[i].astype(np.float32), KEEPS[0])[0], i
        assert seen, "no cohort wait timed out under WC_OPT_SPIN_LIMIT 1"
    finally:
        c.profile_enable(False)
        c.set_option(WC_OPT_SPIN_LIMIT, 0)
        c.set_option(WC_OPT_TICKETS, 0)
        c.set_option(WC_OPT_COHORT, 0)
        c.set_option(WC_OPT_COHORT_LAG, 2)
