"""ctypes binding of the C-ABI in include/wavelet_amd.h (libwavelet_amd.so).

This module is the only place Python touches the native library.  It has no
CPU fallback: loading fails loudly if the shared object is missing, and
creating a context fails loudly if no HIP device is visible.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Iterable, Sequence

import numpy as np

PKG_DIR = Path(__file__).resolve().parent
LIB_DIR = PKG_DIR / "lib"
LIB_PATH = LIB_DIR / "libwavelet_amd.so"
HOST_LIB_PATH = LIB_DIR / "libwavelet_amd_host.so"

WC_OK, WC_ERR_INVALID, WC_ERR_HIP, WC_ERR_NOMEM, WC_ERR_FORMAT = 0, 1, 2, 3, 4
WC_F32, WC_F64 = 0, 1

# Every symbol include/wavelet_amd.h declares (checked by tests/test_capi.py).
EXPORTED = (
    "wc_ctx_create", "wc_ctx_destroy", "wc_last_error", "wc_set_stream", "wc_synchronize",
    "wc_payload_bound", "wc_cell_count", "wc_forward", "wc_forward_host", "wc_decompose",
    "wc_inverse", "wc_inverse_host", "wc_inverse_flat", "wc_rmse", "wc_version",
    "wc_profile_enable", "wc_profile_read", "wc_set_option", "wc_inverse_flat_host", "wc_rmse_host",
    "wc_decompose_host", "wc_device_count", "wc_forward_stage", "wc_hist_threshold",
    "wc_forward_emit", "wc_inverse_rmse", "wc_get_option", "wc_rowindex_bytes", "wc_forward_rows",
    "wc_inverse_rows", "wc_forward_host_units", "wc_round_trip_host",
)
WC_OPT_SPARSE = 12   # sparse coefficient staging in the forward (default 1)
WC_OPT_ORDERED = 13  # look-back tile index from the launch order (1, default) or per-unit tickets (0)
WC_OPT_INVERSE_ROWS = 14  # row-indexed inverse of even-dims units (1, default) or dense decode (0)
WC_OPT_RIX_LDS = 15  # row-indexed inverse: LDS floats per workgroup (default 9216)
WC_OPT_RIX_TX = 16  # row-indexed inverse: log2 of the tile's x blocks (default 4)
WC_OPT_RIX_BLOCKED = 17  # row-indexed inverse: contiguous tile runs per workgroup (default 0)
WC_OPT_HOST_CHUNK = 18  # wc_forward_host: cells per pipelined unit run (default 2^25, 0 = one run)
WC_OPT_SPIN_LIMIT = 19  # polls of an unpublished look-back predecessor before a block derives it itself (0: 64)
WC_OPT_TICKETS = 20  # 1: ticket form whatever WC_OPT_ORDERED says
WC_OPT_REVERSE_TILES = 29  # test hook: each unit's look-back tiles in reverse launch order
WC_OPT_RIX_XCD = 22  # row-indexed inverse tiles dealt to XCDs in contiguous runs (default 0)
WC_OPT_INV_GROUPS = 23  # row-indexed inverse in N unit groups, row index of g+1 beside K6r of g (default 1)
WC_OPT_HOST_THREADS = 27  # _host calls: threads that fault in a copy's host destination first (0 = off)
WC_OPT_HOST_THP = 28  # _host calls: advise huge pages on those destinations (default 0)

# Stage ids of wc_profile_read (include/wavelet_amd.h WC_STAGE_*).
STAGES = ("transform", "emit", "decode", "inverse", "rmse", "hist", "pairs")


class WcUnit(ctypes.Structure):
    """wc_unit: one Box3D component, x fastest (reference src/grid.h:15-19)."""
    _fields_ = [("cell_offset", ctypes.c_uint64), ("nx", ctypes.c_int32),
                ("ny", ctypes.c_int32), ("nz", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class WaveletError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"wavelet_amd error {code}: {msg}")
        self.code = code


_lib = None


def load_library() -> ctypes.CDLL:
    """Load libwavelet_amd.so (built by __graft_entry__.build()); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise FileNotFoundError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    _share_torch_runtime()
    # WCAMD_LIB: another build of the same library (A/B runs of kernel variants)
    L = ctypes.CDLL(os.environ.get("WCAMD_LIB") or str(LIB_PATH))
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    up = ctypes.POINTER(WcUnit)
    sigs = {
        "wc_ctx_create": (i32, [i32, ctypes.POINTER(vp)]),
        "wc_ctx_destroy": (None, [vp]),
        "wc_last_error": (ctypes.c_char_p, [vp]),
        "wc_set_stream": (i32, [vp, vp]),
        "wc_synchronize": (i32, [vp]),
        "wc_payload_bound": (u64, [up, i32]),
        "wc_cell_count": (u64, [up, i32]),
        "wc_forward": (i32, [vp, vp, i32, up, i32, ctypes.c_double, vp, u64, vp, vp]),
        "wc_forward_host": (i32, [vp, vp, i32, up, i32, ctypes.c_double, vp, u64, vp, vp]),
        "wc_decompose": (i32, [vp, vp, i32, up, i32, vp]),
        "wc_inverse": (i32, [vp, vp, vp, up, i32, vp]),
        "wc_inverse_host": (i32, [vp, vp, vp, up, i32, vp]),
        "wc_inverse_flat": (i32, [vp, vp, up, i32, vp]),
        "wc_inverse_rmse": (i32, [vp, vp, vp, up, i32, vp, i32, vp, vp]),
        "wc_rmse": (i32, [vp, vp, i32, vp, up, i32, vp]),
        "wc_version": (ctypes.c_char_p, []),
        "wc_profile_enable": (i32, [vp, i32]),
        "wc_set_option": (i32, [vp, i32, ctypes.c_int64]),
        "wc_get_option": (i32, [vp, i32, ctypes.POINTER(ctypes.c_int64)]),
        "wc_inverse_flat_host": (i32, [vp, vp, up, i32, vp]),
        "wc_rmse_host": (i32, [vp, vp, i32, vp, up, i32, vp]),
        "wc_decompose_host": (i32, [vp, vp, i32, up, i32, vp]),
        "wc_profile_read": (i32, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32), i32]),
        "wc_forward_stage": (i32, [vp, vp, i32, up, i32, vp]),
        "wc_hist_threshold": (i32, [vp, ctypes.c_double, ctypes.POINTER(ctypes.c_float),
                                    ctypes.POINTER(ctypes.c_uint64)]),
        "wc_forward_emit": (i32, [vp, up, i32, ctypes.c_double, ctypes.POINTER(ctypes.c_float), vp, u64,
                                  vp, vp]),
        "wc_rowindex_bytes": (u64, [up, i32]),
        "wc_forward_rows": (i32, [vp, vp, i32, up, i32, ctypes.c_double, vp, u64, vp, vp, vp, u64]),
        "wc_inverse_rows": (i32, [vp, vp, vp, up, i32, vp, u64, vp, i32, vp, vp]),
        "wc_forward_host_units": (i32, [vp, ctypes.POINTER(vp), i32, up, i32, ctypes.c_double, vp, u64, vp, vp]),
        "wc_round_trip_host": (i32, [vp, vp, i32, up, i32, ctypes.c_double, vp, u64, vp, vp, vp]),
    }
    for name, (res, args) in sigs.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def make_units(dims: Sequence[Sequence[int]], offsets: Iterable[int] | None = None,
               align: int = 4):
    """Build a wc_unit array for boxes of `dims` = [(W, H, D), ...].

    Without explicit offsets the boxes are packed back to back, each start
    rounded up to `align` elements (vector loads stay aligned)."""
    n = len(dims)
    arr = (WcUnit * max(n, 1))()
    cur = 0
    offs = list(offsets) if offsets is not None else None
    for i, (W, H, D) in enumerate(dims):
        if offs is None:
            cur = (cur + align - 1) // align * align
            off = cur
            cur += W * H * D
        else:
            off = offs[i]
        arr[i] = WcUnit(off, W, H, D, 0)
    extent = max((arr[i].cell_offset + arr[i].nx * arr[i].ny * arr[i].nz for i in range(n)), default=0)
    return arr, n, int(extent)


def payload_bound(units, n) -> int:
    return int(load_library().wc_payload_bound(units, n))


def rowindex_bytes(units, n) -> int:
    """Bytes of a batch's row index (wc_rowindex_bytes: W*H + 1 entries of 8 B per unit
    with cells, none for an empty unit)."""
    return int(load_library().wc_rowindex_bytes(units, n))


def _share_torch_runtime():
    """torch ships its own HIP runtime (torch/lib/libamdhip64.so, SONAME
    libamdhip64.so.7, ROCm 7.0) beside the system one this library links
    (/opt/rocm/lib/libamdhip64.so.7).  If torch is loaded first, the dynamic
    loader resolves our NEEDED libamdhip64.so.7 to torch's copy and the process
    has ONE HIP runtime; loaded the other way round there would be two, and
    only the first to initialise gets the GPU.  So import torch (if present)
    before dlopen-ing the library.  Set WCAMD_NO_TORCH=1 to skip (torch-free
    processes then use the system ROCm runtime)."""
    if os.environ.get("WCAMD_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


class Context:
    """One wc_ctx: a HIP device, its stream and its HBM scratch."""

    def __init__(self, device: int = 0):
        L = load_library()
        h = ctypes.c_void_p()
        rc = L.wc_ctx_create(int(device), ctypes.byref(h))
        if rc != WC_OK:
            raise WaveletError(rc, f"wc_ctx_create(device={device}) failed: no usable HIP device")
        self._h = h
        self.device = device
        self._L = L

    def close(self):
        if self._h:
            self._L.wc_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int):
        if rc != WC_OK:
            raise WaveletError(rc, self._L.wc_last_error(self._h).decode())

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: int | None):
        self._check(self._L.wc_set_stream(self._h, ctypes.c_void_p(stream_ptr or 0)))

    def synchronize(self):
        self._check(self._L.wc_synchronize(self._h))

    def set_option(self, option: int, value: int):
        self._check(self._L.wc_set_option(self._h, int(option), int(value)))

    def get_option(self, option: int) -> int:
        v = ctypes.c_int64()
        self._check(self._L.wc_get_option(self._h, int(option), ctypes.byref(v)))
        return int(v.value)

    def profile_enable(self, on: bool = True):
        self._check(self._L.wc_profile_enable(self._h, 1 if on else 0))

    def profile_read(self) -> dict:
        """{stage: (total_ms, launches)} since the previous read (hipEvent timing)."""
        n = len(STAGES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_uint32 * n)()
        self._check(self._L.wc_profile_read(self._h, ms, cnt, n))
        return {STAGES[i]: (ms[i], cnt[i]) for i in range(n) if cnt[i]}

    # ---- device-pointer API (torch tensors or raw ints) ------------------
    def forward(self, d_cells: int, dtype: int, units, n: int, keep: float, d_payload: int,
                capacity: int, d_offsets: int, d_kept: int):
        self._check(self._L.wc_forward(self._h, ctypes.c_void_p(d_cells), dtype, units, n,
                                       float(keep), ctypes.c_void_p(d_payload), capacity,
                                       ctypes.c_void_p(d_offsets), ctypes.c_void_p(d_kept)))

    def forward_rows(self, d_cells: int, dtype: int, units, n: int, keep: float, d_payload: int,
                     capacity: int, d_offsets: int, d_kept: int, d_rowinfo: int, rowinfo_capacity: int):
        """wc_forward that also writes the payloads' row index (include/wavelet_amd.h)."""
        self._check(self._L.wc_forward_rows(self._h, ctypes.c_void_p(d_cells), dtype, units, n, float(keep),
                                            ctypes.c_void_p(d_payload), capacity, ctypes.c_void_p(d_offsets),
                                            ctypes.c_void_p(d_kept), ctypes.c_void_p(d_rowinfo), rowinfo_capacity))

    def inverse_rows(self, d_payload: int, d_offsets: int, units, n: int, d_rowinfo: int | None, d_out: int,
                     d_orig: int | None = None, dtype: int = WC_F32, d_rmse: int | None = None,
                     rowinfo_capacity: int | None = None):
        """wc_inverse (d_orig None) or wc_inverse_rmse with the row index of
        wc_forward_rows (d_rowinfo None: derived from the payloads).
        rowinfo_capacity: bytes of the d_rowinfo buffer (default: exactly
        rowindex_bytes(units, n), the size forward_rows needs)."""
        cap = rowinfo_capacity if rowinfo_capacity is not None else (rowindex_bytes(units, n) if d_rowinfo else 0)
        self._check(self._L.wc_inverse_rows(self._h, ctypes.c_void_p(d_payload), ctypes.c_void_p(d_offsets),
                                            units, n, ctypes.c_void_p(d_rowinfo or 0), cap,
                                            ctypes.c_void_p(d_orig or 0), dtype, ctypes.c_void_p(d_out),
                                            ctypes.c_void_p(d_rmse or 0)))

    def forward_stage(self, d_cells: int, dtype: int, units, n: int, d_hist: int | None = None):
        """Global-threshold mode, step 1 (include/wavelet_amd.h): transform into
        the context scratch; add the magnitude histogram to d_hist if given."""
        self._check(self._L.wc_forward_stage(self._h, ctypes.c_void_p(d_cells), dtype, units, n,
                                             ctypes.c_void_p(d_hist or 0)))

    def forward_emit(self, units, n: int, keep: float, thresh: float | None, d_payload: int,
                     capacity: int, d_offsets: int, d_kept: int):
        """Step 2: pack the staged batch with one fp32 threshold (None: the
        reference's per-unit rule with `keep`)."""
        t = None if thresh is None else ctypes.byref(ctypes.c_float(thresh))
        self._check(self._L.wc_forward_emit(self._h, units, n, float(keep), t, ctypes.c_void_p(d_payload),
                                            capacity, ctypes.c_void_p(d_offsets), ctypes.c_void_p(d_kept)))

    def decompose(self, d_cells: int, dtype: int, units, n: int, d_flat: int):
        self._check(self._L.wc_decompose(self._h, ctypes.c_void_p(d_cells), dtype, units, n,
                                         ctypes.c_void_p(d_flat)))

    def inverse(self, d_payload: int, d_offsets: int, units, n: int, d_out: int):
        self._check(self._L.wc_inverse(self._h, ctypes.c_void_p(d_payload), ctypes.c_void_p(d_offsets),
                                       units, n, ctypes.c_void_p(d_out)))

    def inverse_rmse(self, d_payload: int, d_offsets: int, units, n: int, d_orig: int, dtype: int, d_out: int,
                     d_rmse: int):
        """inverse + rmse fused (include/wavelet_amd.h wc_inverse_rmse)."""
        self._check(self._L.wc_inverse_rmse(self._h, ctypes.c_void_p(d_payload), ctypes.c_void_p(d_offsets),
                                            units, n, ctypes.c_void_p(d_orig), dtype, ctypes.c_void_p(d_out),
                                            ctypes.c_void_p(d_rmse)))

    def inverse_flat(self, d_flat: int, units, n: int, d_out: int):
        self._check(self._L.wc_inverse_flat(self._h, ctypes.c_void_p(d_flat), units, n,
                                            ctypes.c_void_p(d_out)))

    def rmse(self, d_orig: int, dtype: int, d_regen: int, units, n: int, d_rmse: int):
        self._check(self._L.wc_rmse(self._h, ctypes.c_void_p(d_orig), dtype, ctypes.c_void_p(d_regen),
                                    units, n, ctypes.c_void_p(d_rmse)))

    # ---- host-array API ---------------------------------------------------
    def forward_host(self, cells: np.ndarray, units, n: int, keep: float, out=None):
        """cells: flat host array (float32 or float64) -> (payload bytes, offsets, kept).
        out: optional (payload uint8[>= payload_bound], offsets uint64[n + 1],
        kept uint32[>= n]) to fill instead of new arrays (a caller that streams
        batches reuses its buffers: no page faults, no frees per call)."""
        c = np.ascontiguousarray(cells)
        dtype = WC_F64 if c.dtype == np.float64 else WC_F32
        if c.dtype not in (np.float32, np.float64):
            raise TypeError("cells must be float32 or float64")
        cap = payload_bound(units, n)
        if out is None:
            payload = np.empty(cap, np.uint8)
            offsets = np.zeros(n + 1, np.uint64)
            kept = np.zeros(max(n, 1), np.uint32)
        else:
            payload, offsets, kept = out
            if (payload.dtype != np.uint8 or payload.size < cap or not payload.flags.c_contiguous
                    or offsets.dtype != np.uint64 or offsets.size < n + 1 or not offsets.flags.c_contiguous
                    or kept.dtype != np.uint32 or kept.size < n or not kept.flags.c_contiguous):
                raise ValueError("out: (uint8[>= payload_bound], uint64[n + 1], uint32[n]) contiguous arrays")
            cap = payload.size
        self._check(self._L.wc_forward_host(self._h, c.ctypes.data, dtype, units, n, float(keep),
                                            payload.ctypes.data, cap, offsets.ctypes.data,
                                            kept.ctypes.data))
        return payload, offsets, kept[:n]

    def round_trip_host(self, cells: np.ndarray, units, n: int, keep: float):
        """wc_round_trip_host: forward_host's (payload, offsets, kept) and the
        per-unit RMSE of the reconstruction (computed on the device)."""
        c = np.ascontiguousarray(cells)
        if c.dtype not in (np.float32, np.float64):
            raise TypeError("cells must be float32 or float64")
        dtype = WC_F64 if c.dtype == np.float64 else WC_F32
        cap = payload_bound(units, n)
        payload = np.empty(cap, np.uint8)
        offsets = np.zeros(n + 1, np.uint64)
        kept = np.zeros(max(n, 1), np.uint32)
        rmse = np.zeros(max(n, 1), np.float64)
        self._check(self._L.wc_round_trip_host(self._h, c.ctypes.data, dtype, units, n, float(keep),
                                               payload.ctypes.data, cap, offsets.ctypes.data, kept.ctypes.data,
                                               rmse.ctypes.data))
        return payload, offsets, kept[:n], rmse[:n]

    def forward_host_units(self, boxes, units, n: int, keep: float):
        """wc_forward_host_units: unit u's cells from boxes[u] (its own host
        array, all float32 or all float64) -> (payload, offsets, kept)."""
        arrs = [np.ascontiguousarray(b) for b in boxes]
        dt = {a.dtype for a in arrs if a.size}
        if not dt <= {np.dtype(np.float32)} and not dt <= {np.dtype(np.float64)}:
            raise TypeError("boxes must be all float32 or all float64")
        dtype = WC_F64 if dt == {np.dtype(np.float64)} else WC_F32
        ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
        cap = payload_bound(units, n)
        payload = np.empty(cap, np.uint8)
        offsets = np.zeros(n + 1, np.uint64)
        kept = np.zeros(max(n, 1), np.uint32)
        self._check(self._L.wc_forward_host_units(self._h, ptrs, dtype, units, n, float(keep), payload.ctypes.data,
                                                  cap, offsets.ctypes.data, kept.ctypes.data))
        return payload, offsets, kept[:n]

    def decompose_host(self, cells: np.ndarray, units, n: int, extent: int) -> np.ndarray:
        c = np.ascontiguousarray(cells)
        dtype = WC_F64 if c.dtype == np.float64 else WC_F32
        out = np.zeros(max(extent, 1), np.float32)
        self._check(self._L.wc_decompose_host(self._h, c.ctypes.data, dtype, units, n, out.ctypes.data))
        return out[:extent]

    def inverse_flat_host(self, flat: np.ndarray, units, n: int, extent: int) -> np.ndarray:
        f = np.ascontiguousarray(flat, np.float32)
        out = np.zeros(max(extent, 1), np.float32)
        self._check(self._L.wc_inverse_flat_host(self._h, f.ctypes.data, units, n, out.ctypes.data))
        return out[:extent]

    def rmse_host(self, orig: np.ndarray, regen: np.ndarray, units, n: int) -> np.ndarray:
        o = np.ascontiguousarray(orig)
        dtype = WC_F64 if o.dtype == np.float64 else WC_F32
        r = np.ascontiguousarray(regen, np.float32)
        out = np.zeros(max(n, 1), np.float64)
        self._check(self._L.wc_rmse_host(self._h, o.ctypes.data, dtype, r.ctypes.data, units, n, out.ctypes.data))
        return out[:n]

    def inverse_host(self, payload: np.ndarray, offsets: np.ndarray, units, n: int, extent: int, out=None):
        """-> float32[extent] boxes (cells no unit owns stay 0, or as they were in `out`)."""
        p = np.ascontiguousarray(payload, dtype=np.uint8)
        o = np.ascontiguousarray(offsets, dtype=np.uint64)
        if out is None:
            out = np.zeros(max(extent, 1), np.float32)
        elif out.dtype != np.float32 or out.size < extent or not out.flags.c_contiguous:
            raise ValueError("out: contiguous float32[>= extent]")
        self._check(self._L.wc_inverse_host(self._h, p.ctypes.data, o.ctypes.data, units, n,
                                            out.ctypes.data))
        return out[:extent]


HIST_BINS = 4096  # WC_HIST_BINS
HIST_SHIFT = 19   # WC_HIST_SHIFT


def hist_threshold(hist: np.ndarray, quantile: float):
    """wc_hist_threshold (host only): (fp32 threshold, retained count) for an
    all-reduced WC_HIST_BINS uint64 histogram."""
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    if h.size != HIST_BINS:
        raise ValueError(f"histogram must have {HIST_BINS} bins")
    t = ctypes.c_float()
    r = ctypes.c_uint64()
    rc = load_library().wc_hist_threshold(h.ctypes.data, float(quantile), ctypes.byref(t), ctypes.byref(r))
    if rc:
        raise WaveletError(rc, "wc_hist_threshold: invalid argument")
    return float(t.value), int(r.value)


def unit_payload(payload: np.ndarray, offsets: np.ndarray, kept: np.ndarray, u: int) -> bytes:
    """Unit u's serialized bytes (reference src/compressor.cpp:55-80 layout)."""
    o = int(offsets[u])
    return payload[o:o + 20 + 8 * int(kept[u])].tobytes()
