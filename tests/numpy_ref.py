"""A second, independent restatement of the reference transform in numpy.

Test infrastructure: it cross-checks the C oracle (oracle/wc_oracle.c) with
whole-axis array operations instead of per-line loops, following the same
reference semantics (src/compressor.cpp:85-185, src/decompressor.cpp:79-159):
float32 pair sums, exact halving, one rounding; inverse sums in float64 then
narrowed; odd tails pass through forward and come back as 0.
Boxes are numpy arrays of shape (D, H, W) (x fastest).
"""
import numpy as np


def _fwd_axis(a: np.ndarray, axis: int) -> np.ndarray:
    n = a.shape[axis]
    h = n // 2
    x = np.moveaxis(a, axis, 0)
    even, odd = x[0:2 * h:2], x[1:2 * h:2]
    s = (even + odd).astype(np.float64) / 2.0   # float add, exact halving
    d = (even - odd).astype(np.float64) / 2.0
    parts = [s.astype(np.float32), d.astype(np.float32)]
    if n % 2:
        parts.append(x[2 * h:])
    return np.moveaxis(np.concatenate(parts, axis=0), 0, axis)


def wavelet_decompose(box: np.ndarray) -> np.ndarray:
    b = np.asarray(box, np.float32)
    b = _fwd_axis(b, 0)   # Z sweep first
    b = _fwd_axis(b, 1)   # then Y
    b = _fwd_axis(b, 2)   # then X
    return np.ascontiguousarray(np.transpose(b, (2, 1, 0))).ravel()  # (x, y, z) order, z fastest


def _inv_axis(a: np.ndarray, axis: int) -> np.ndarray:
    n = a.shape[axis]
    h = n // 2
    x = np.moveaxis(a, axis, 0).astype(np.float64)
    avg, diff = x[0:h], x[h:2 * h]
    out = np.zeros_like(x)
    out[0:2 * h:2] = avg + diff
    out[1:2 * h:2] = avg - diff
    return np.moveaxis(out.astype(np.float32), 0, axis)


def inverse_wavelet_decompose(flat: np.ndarray, W: int, H: int, D: int) -> np.ndarray:
    b = np.asarray(flat, np.float32).reshape(W, H, D).transpose(2, 1, 0)  # back to (z, y, x)
    b = _inv_axis(b, 2)   # X first
    b = _inv_axis(b, 1)   # then Y
    b = _inv_axis(b, 0)   # then Z
    return np.ascontiguousarray(b)


def compress_payload(box: np.ndarray, keep: float) -> bytes:
    flat = wavelet_decompose(box)
    n = flat.size
    if n == 0:
        D, H, W = box.shape
        return np.array([W, H, D, 0, 0], "<i4").tobytes()
    mags = np.abs(flat.astype(np.float64))
    # std::max_element semantics: first index of the largest |c|; NaN only if flat[0] is NaN
    if np.isnan(flat[0]):
        thresh = np.nan
    else:
        m = np.where(np.isnan(mags), -1.0, mags)
        idx = int(np.argmax(m))
        thresh = float(flat[idx]) * (1 - keep)
    mask = mags > thresh
    pos = np.flatnonzero(mask)
    runs = np.diff(np.concatenate([[-1], pos])) - 1
    D, H, W = box.shape
    hdr = np.array([W, H, D, n, pos.size], "<i4").tobytes()
    pairs = np.empty(pos.size, dtype=[("r", "<i4"), ("v", "<f4")])
    pairs["r"] = runs
    pairs["v"] = flat[pos]
    return hdr + pairs.tobytes()


def row_index(payload: bytes, W: int, H: int, D: int) -> np.ndarray:
    """The row index of one payload (include/wavelet_amd.h wc_rowindex_bytes):
    (W*H + 1, 2) uint32, entry r = (k, p_k - r*D), k the first pair whose flat
    position p_k (rle_decode's idx, src/decompressor.cpp:14-30) is >= r*D, or
    (nrle, ncoeff - r*D) past the last pair."""
    hdr = np.frombuffer(payload[:20], "<i4")
    n, nrle = int(hdr[3]), int(hdr[4])
    pairs = np.frombuffer(payload[20:20 + 8 * nrle], dtype=[("r", "<i4"), ("v", "<f4")])
    pos = np.cumsum(pairs["r"].astype(np.int64) + 1) - 1
    starts = np.arange(W * H + 1, dtype=np.int64) * D
    k = np.searchsorted(pos, starts, side="left")
    p = np.where(k < nrle, pos[np.minimum(k, max(nrle - 1, 0))] if nrle else n, n)
    return np.stack([k, p - starts], axis=1).astype(np.uint32)
