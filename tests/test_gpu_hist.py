"""GPU: the opt-in global-threshold mode (include/wavelet_amd.h wc_forward_stage /
wc_hist_threshold / wc_forward_emit) against the oracle restatement.

Bar: the device histogram equals the oracle's bin counts exactly; stage + emit
with no threshold is byte-identical to wc_forward (the reference rule); stage +
emit with a global threshold is byte-identical to the reference's mask + RLE +
serialize applied with that threshold (oracle.compress_payload_thresh), and the
kept total equals the histogram's retained count.
"""
import numpy as np
import pytest

from test_gpu_parity import DIMS, pack, synth

pytestmark = pytest.mark.gpu


def _run(wc, ctx, cells, units, n, extent, keep, quantiles):
    import torch
    dev = torch.device("cuda", 0)
    dtype = wc.capi.WC_F64 if cells.dtype == np.float64 else wc.capi.WC_F32
    d_cells = torch.from_numpy(cells).to(dev)
    hist = torch.zeros(wc.capi.HIST_BINS, dtype=torch.int64, device=dev)
    cap = wc.capi.payload_bound(units, n)
    d_pay = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.forward_stage(d_cells.data_ptr(), dtype, units, n, hist.data_ptr())
    ctx.synchronize()
    h = hist.cpu().numpy().view(np.uint64).copy()

    def emit(thresh):
        ctx.forward_emit(units, n, keep, thresh, d_pay.data_ptr(), cap, d_off.data_ptr(), d_kept.data_ptr())
        ctx.synchronize()
        pay = d_pay.cpu().numpy()
        off = d_off.cpu().numpy().view(np.uint64)
        kept = d_kept.cpu().numpy().view(np.uint32)
        return [wc.capi.unit_payload(pay, off, kept, i) for i in range(n)], kept

    out = {"hist": h, None: emit(None)}
    for q in quantiles:
        t, r = wc.capi.hist_threshold(h, q)
        out[q] = (t, r, emit(t))  # the staged coefficients are reused for every threshold
    return out


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_histogram_mode_bit_exact(wc, ctx, oracle, dtype):
    keep = float(np.float32(0.999))
    boxes = synth(oracle, DIMS, seed0=3)
    units, n, extent, cells = pack(wc, boxes, dtype)
    quantiles = (0.0, 0.5, 0.9, 0.999, 1.0)
    out = _run(wc, ctx, cells, units, n, extent, keep, quantiles)
    b32 = [oracle.narrow(b) for b in boxes]
    flats = [oracle.wavelet_decompose(b) for b in b32]
    want_h = sum(oracle.magnitude_hist(f) for f in flats)
    assert np.array_equal(out["hist"], want_h)
    ref_payloads, _ = out[None]
    for i, b in enumerate(b32):
        assert ref_payloads[i] == oracle.compress_payload(b, keep)[0], f"unit {i} reference rule"
    for q in quantiles:
        t, r, (payloads, kept) = out[q]
        assert (t, r) == oracle.hist_threshold(want_h, q)
        assert int(kept.sum()) == r
        for i, b in enumerate(b32):
            assert payloads[i] == oracle.compress_payload_thresh(b, t), f"unit {i} dims {DIMS[i]} q {q}"


def test_histogram_mode_round_trip_64cubed(wc, ctx, oracle):
    """64 boxes of 64^3 fp64: global threshold at the median, payloads decode
    through the unchanged inverse path to the oracle's reconstruction."""
    boxes = [oracle.synth_box_f64(oracle.unit_seed(0, 0, i, 0), (64 * i, 0, 0), 64, 64, 64) for i in range(64)]
    units, n, extent, cells = pack(wc, boxes, np.float64)
    out = _run(wc, ctx, cells, units, n, extent, 0.999, (0.5,))
    t, r, (payloads, kept) = out[0.5]
    assert r >= (n * 64 ** 3) // 2 and int(kept.sum()) == r
    for i in (0, 17, 63):
        assert payloads[i] == oracle.compress_payload_thresh(oracle.narrow(boxes[i]), t)
    blob = np.frombuffer(b"".join(payloads), np.uint8)
    offs = np.cumsum([0] + [len(p) for p in payloads]).astype(np.uint64)
    regen = ctx.inverse_host(blob, offs, units, n, extent)
    for i in (0, 63):
        o = units[i].cell_offset
        ref = oracle.decompress_payload(payloads[i]).ravel()
        assert regen[o:o + ref.size].tobytes() == ref.tobytes()


def test_emit_without_stage_is_rejected(wc, ctx, oracle):
    import torch
    boxes = synth(oracle, DIMS[:3])
    units, n, extent, cells = pack(wc, boxes)
    cap = wc.capi.payload_bound(units, n)
    dev = torch.device("cuda", 0)
    d_pay = torch.empty(cap, dtype=torch.uint8, device=dev)
    d_off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    d_kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # the fills above run on torch's stream, the context on its own
    ctx.forward_host(cells, units, n, 0.999)  # any other call invalidates the staged scratch
    with pytest.raises(wc.WaveletError):
        ctx.forward_emit(units, n, 0.999, None, d_pay.data_ptr(), cap, d_off.data_ptr(), d_kept.data_ptr())
