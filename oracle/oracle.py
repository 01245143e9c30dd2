"""Python handle on the CPU oracle (oracle/wc_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  Every function is
a thin numpy wrapper over the C restatement, which cites the reference
file:line it follows (carsonmw3/wavelet-compression src/compressor.cpp,
src/decompressor.cpp, src/calc-loss.cpp).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "build" / "liboracle.so"

_lib = None


def build() -> Path:
    """Compile the oracle with its Makefile (gcc, no fast-math)."""
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = ctypes.CDLL(str(LIB_PATH))
        f32p = ctypes.POINTER(ctypes.c_float)
        f64p = ctypes.POINTER(ctypes.c_double)
        i32p = ctypes.POINTER(ctypes.c_int32)
        i64p = ctypes.POINTER(ctypes.c_int64)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        i32, i64, dbl = ctypes.c_int, ctypes.c_int64, ctypes.c_double
        sig = {
            "wco_narrow_f64": (None, [f64p, f32p, i64]),
            "wco_wavelet_decompose": (None, [f32p, i32, i32, i32, f32p]),
            "wco_max_index": (i64, [f32p, i64]),
            "wco_threshold": (dbl, [f32p, i64, dbl]),
            "wco_threshold_rle": (i64, [f32p, i64, dbl, i32p, f32p]),
            "wco_rle_encode": (i64, [u8p, f32p, i64, i32p, f32p]),
            "wco_serialized_size": (ctypes.c_size_t, [i64]),
            "wco_serialize": (ctypes.c_size_t, [i32, i32, i32, ctypes.c_int32, i64, i32p, f32p, u8p]),
            "wco_compress_payload": (ctypes.c_size_t, [f32p, i32, i32, i32, dbl, u8p, i64p]),
            "wco_rle_decode": (None, [i32p, f32p, i64, i64, f32p]),
            "wco_payload_to_flat": (ctypes.c_int, [u8p, ctypes.c_size_t, f32p, i64]),
            "wco_inverse_wavelet_decompose": (None, [f32p, i32, i32, i32, f32p]),
            "wco_rmse": (dbl, [f32p, f32p, i32, i32, i32]),
            "wco_synth_box_f64": (None, [ctypes.c_uint64, i32, i32, i32, i32, i32, i32, dbl, f64p]),
            "wco_unit_seed": (ctypes.c_uint64, [i32, i32, i32, i32]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _p(a: np.ndarray, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


def _box_dims(box: np.ndarray):
    """Box3D arrays are numpy [D, H, W] (z slowest) so that x is fastest."""
    D, H, W = box.shape
    return W, H, D


def narrow(cells64: np.ndarray) -> np.ndarray:
    c = np.ascontiguousarray(cells64, dtype=np.float64)
    out = np.empty(c.shape, np.float32)
    lib().wco_narrow_f64(_p(c, ctypes.c_double), _p(out, ctypes.c_float), c.size)
    return out


def wavelet_decompose(box: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(box, dtype=np.float32)
    W, H, D = _box_dims(b)
    flat = np.empty(W * H * D, np.float32)
    lib().wco_wavelet_decompose(_p(b, ctypes.c_float), W, H, D, _p(flat, ctypes.c_float))
    return flat


def max_index(flat: np.ndarray) -> int:
    f = np.ascontiguousarray(flat, dtype=np.float32)
    return int(lib().wco_max_index(_p(f, ctypes.c_float), f.size))


def threshold(flat: np.ndarray, keep: float) -> float:
    f = np.ascontiguousarray(flat, dtype=np.float32)
    return float(lib().wco_threshold(_p(f, ctypes.c_float), f.size, float(keep)))


def threshold_rle(flat: np.ndarray, thresh: float):
    f = np.ascontiguousarray(flat, dtype=np.float32)
    runs = np.empty(max(f.size, 1), np.int32)
    vals = np.empty(max(f.size, 1), np.float32)
    n = lib().wco_threshold_rle(_p(f, ctypes.c_float), f.size, float(thresh),
                                _p(runs, ctypes.c_int32), _p(vals, ctypes.c_float))
    return runs[:n].copy(), vals[:n].copy()


def rle_encode(mask, values):
    m = np.ascontiguousarray(mask, dtype=np.uint8)
    v = np.ascontiguousarray(values, dtype=np.float32)
    runs = np.empty(max(m.size, 1), np.int32)
    vals = np.empty(max(m.size, 1), np.float32)
    n = lib().wco_rle_encode(_p(m, ctypes.c_uint8), _p(v, ctypes.c_float), m.size,
                             _p(runs, ctypes.c_int32), _p(vals, ctypes.c_float))
    return list(zip(runs[:n].tolist(), vals[:n].tolist()))


def serialize(W, H, D, ncoeff, runs, vals) -> bytes:
    r = np.ascontiguousarray(runs, dtype=np.int32)
    v = np.ascontiguousarray(vals, dtype=np.float32)
    out = np.empty(lib().wco_serialized_size(r.size), np.uint8)
    n = lib().wco_serialize(W, H, D, ncoeff, r.size, _p(r, ctypes.c_int32),
                            _p(v, ctypes.c_float), _p(out, ctypes.c_uint8))
    return out[:n].tobytes()


def compress_payload(box: np.ndarray, keep: float):
    """compress() for one component minus xz -> (payload bytes, kept)."""
    b = np.ascontiguousarray(box, dtype=np.float32)
    W, H, D = _box_dims(b)
    out = np.empty(lib().wco_serialized_size(W * H * D), np.uint8)
    kept = ctypes.c_int64(0)
    n = lib().wco_compress_payload(_p(b, ctypes.c_float), W, H, D, float(keep),
                                   _p(out, ctypes.c_uint8), ctypes.byref(kept))
    return out[:n].tobytes(), int(kept.value)


def parse_payload(payload: bytes):
    """deserialize_compressed_wavelet -> (shape, ncoeff, runs, vals)."""
    hdr = np.frombuffer(payload[:20], dtype="<i4")
    W, H, D, nc, nr = (int(x) for x in hdr)
    body = np.frombuffer(payload[20:20 + 8 * nr], dtype=np.uint8)
    pairs = body.view(np.int32).reshape(-1, 2)
    runs = pairs[:, 0].copy()
    vals = pairs[:, 1].copy().view(np.float32)
    return (W, H, D), nc, runs, vals


def rle_decode(runs, vals, total: int) -> np.ndarray:
    r = np.ascontiguousarray(runs, dtype=np.int32)
    v = np.ascontiguousarray(vals, dtype=np.float32)
    out = np.empty(max(total, 1), np.float32)
    lib().wco_rle_decode(_p(r, ctypes.c_int32), _p(v, ctypes.c_float), r.size, total,
                         _p(out, ctypes.c_float))
    return out[:total]


def inverse_wavelet_decompose(flat: np.ndarray, W: int, H: int, D: int) -> np.ndarray:
    f = np.ascontiguousarray(flat, dtype=np.float32)
    box = np.empty((D, H, W), np.float32)
    lib().wco_inverse_wavelet_decompose(_p(f, ctypes.c_float), W, H, D, _p(box, ctypes.c_float))
    return box


def decompress_payload(payload: bytes) -> np.ndarray:
    """decompress() minus xz: payload -> rle_decode -> inverse (Box3D [D,H,W])."""
    (W, H, D), nc, runs, vals = parse_payload(payload)
    flat = rle_decode(runs, vals, nc)
    return inverse_wavelet_decompose(flat, W, H, D)


def rmse(actual: np.ndarray, pred: np.ndarray) -> float:
    a = np.ascontiguousarray(actual, dtype=np.float32)
    p = np.ascontiguousarray(pred, dtype=np.float32)
    W, H, D = _box_dims(a)
    return float(lib().wco_rmse(_p(a, ctypes.c_float), _p(p, ctypes.c_float), W, H, D))


def unit_seed(t: int, lev: int, box: int, comp: int) -> int:
    return int(lib().wco_unit_seed(t, lev, box, comp))


def synth_box_f64(seed: int, lo, W: int, H: int, D: int, sigma: float = 0.05) -> np.ndarray:
    out = np.empty((D, H, W), np.float64)
    lib().wco_synth_box_f64(ctypes.c_uint64(seed), int(lo[0]), int(lo[1]), int(lo[2]),
                            W, H, D, float(sigma), _p(out, ctypes.c_double))
    return out


# ---- opt-in global-threshold mode (not the reference's rule) -------------
# numpy restatement of include/wavelet_amd.h's histogram + threshold choice;
# the payload with a given threshold reuses the reference's mask + rle_encode +
# serialize (wco_threshold_rle / wco_serialize: src/compressor.cpp:24-80,222-238)
# with `thresh` in place of max * (1 - keep).
HIST_BINS, HIST_SHIFT = 4096, 19


def magnitude_hist(flat: np.ndarray) -> np.ndarray:
    bits = np.ascontiguousarray(flat, dtype=np.float32).view(np.uint32) & np.uint32(0x7FFFFFFF)
    bits = bits[bits <= 0x7F800000]
    return np.bincount((bits >> HIST_SHIFT).astype(np.int64), minlength=HIST_BINS).astype(np.uint64)


def hist_threshold(hist: np.ndarray, quantile: float):
    """(fp32 threshold, retained) by the rule wc_hist_threshold documents."""
    h = [int(x) for x in hist]
    total = sum(h)
    target = total - min(int(np.floor(quantile * float(total))), total)
    if target == 0:
        return float("inf"), 0
    cum = 0
    for b in range(HIST_BINS - 1, -1, -1):
        cum += h[b]
        if cum >= target:
            if b == 0:
                return -1.0, cum
            return float(np.array([(b << HIST_SHIFT) - 1], np.uint32).view(np.float32)[0]), cum
    return float("inf"), 0


def compress_payload_thresh(box: np.ndarray, thresh: float) -> bytes:
    """One component's payload with an explicit threshold (|c| > thresh kept)."""
    b = np.ascontiguousarray(box, dtype=np.float32)
    W, H, D = _box_dims(b)
    runs, vals = threshold_rle(wavelet_decompose(b), thresh)
    return serialize(W, H, D, W * H * D, runs, vals)
