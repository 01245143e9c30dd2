"""Python mirror of the reference's codec interface, running on the HIP path.

Same names, argument meaning and error behaviour as
carsonmw3/wavelet-compression:

  compress(box, components, keep, time, level, box_index, compressed_dir)
        src/compressor.h:9-15 / src/compressor.cpp:192-297
  decompress(file_path, time, level, component, box_idx)
        src/decompressor.h:6-10 / src/decompressor.cpp:238-255
  deserialize_compressed_wavelet(data)          src/decompressor.h:14, .cpp:35-74
  inverse_wavelet_decompose(flat, x, y, z)      src/decompressor.h:18, .cpp:79-159
  calc_rmse_per_box(actual, pred, num_components) src/calc-loss.h:6-8
  calc_adj_loss(rmse, range)                    src/calc-loss.cpp:49-51
  calc_size(path)                               src/calc-loss.cpp:55-65

A Box3D is a float32 numpy array of shape (D, H, W) — x fastest in memory,
exactly Grid3D's `x + W*(y + H*z)` layout (src/grid.h:15-19).  A multiBox3D
is a list of them.  All transform / threshold / pack / unpack / RMSE work runs
in the HIP kernels; the xz stage is host-side (Python's lzma is liblzma).
"""
from __future__ import annotations

import lzma
import os
import sys
import threading
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Sequence, Tuple

import numpy as np

from . import capi

# Reference: lzma_easy_encoder(&strm, 6, LZMA_CHECK_CRC64) (src/compressor.cpp:261-262)
XZ_PRESET = 6
XZ_CHECK = lzma.CHECK_CRC64


def parse_xz_preset(text: str) -> int:
    """"0".."9", optionally followed by "e" (extreme) -> lzma preset value."""
    t = str(text)
    if len(t) in (1, 2) and t[0].isdigit() and (len(t) == 1 or t[1] == "e"):
        return int(t[0]) | (lzma.PRESET_EXTREME if len(t) == 2 else 0)
    raise ValueError(f"xz preset: 0-9, optionally followed by e, not {text!r}")


def xz_preset() -> int:
    """The preset of compress(): the reference's 6, or $WCAMD_XZ_PRESET (SURVEY
    §8(f) row 1, an optional faster preset; the reference's stream decoder,
    src/decompressor.cpp:189, reads any).  The C++ host library reads the same
    variable (include/wavelet_amd/xz_pool.h)."""
    import os
    v = os.environ.get("WCAMD_XZ_PRESET")
    return XZ_PRESET if not v else parse_xz_preset(v)

_ctx_lock = threading.Lock()
_ctxs: dict = {}


def context(device: int = 0) -> capi.Context:
    """Per-(thread, device) codec context (one wc_ctx per device per host thread)."""
    key = (threading.get_ident(), device)
    with _ctx_lock:
        c = _ctxs.get(key)
        if c is None:
            c = capi.Context(device)
            _ctxs[key] = c
        return c


@dataclass
class CompressedWavelet:
    """src/box-structs.h:65-70."""
    shape: List[int] = field(default_factory=list)          # {W, H, D}
    coeff_shape: List[int] = field(default_factory=list)    # {W*H*D}
    rle_encoded: List[Tuple[int, float]] = field(default_factory=list)
    need32: bool = False

    @property
    def runs(self) -> np.ndarray:
        return np.array([r for r, _ in self.rle_encoded], np.int32)


def _box_dims(b: np.ndarray) -> Tuple[int, int, int]:
    if b.ndim != 3:
        raise ValueError("Box3D must be a 3-D array of shape (D, H, W)")
    D, H, W = b.shape
    return W, H, D


def serialize_compressed_wavelet(cw: CompressedWavelet) -> bytes:
    """src/compressor.cpp:55-80 (static there; exposed here for tests)."""
    hdr = np.array(list(cw.shape) + list(cw.coeff_shape) + [len(cw.rle_encoded)], "<i4").tobytes()
    if not cw.rle_encoded:
        return hdr
    pairs = np.empty(len(cw.rle_encoded), dtype=[("run", "<i4"), ("val", "<f4")])
    pairs["run"] = [r for r, _ in cw.rle_encoded]
    pairs["val"] = [v for _, v in cw.rle_encoded]
    return hdr + pairs.tobytes()


def deserialize_compressed_wavelet(data: bytes) -> CompressedWavelet:
    """src/decompressor.cpp:35-74: 3 dims, 1 coeff dim, pair count, pairs."""
    if len(data) < 20:
        raise ValueError("serialized wavelet shorter than its 20-byte header")
    h = np.frombuffer(data[:20], "<i4")
    nrle = int(h[4])
    if nrle < 0 or len(data) < 20 + 8 * nrle:
        raise ValueError("serialized wavelet truncated")
    pairs = np.frombuffer(data[20:20 + 8 * nrle], dtype=[("run", "<i4"), ("val", "<f4")])
    cw = CompressedWavelet(shape=[int(h[0]), int(h[1]), int(h[2])], coeff_shape=[int(h[3])],
                           rle_encoded=list(zip(pairs["run"].tolist(), pairs["val"].tolist())),
                           need32=False)
    return cw


def _pairs_need32(vals: np.ndarray) -> bool:
    # need32 = any kept |v| > INT16_MAX (src/compressor.cpp:229); never serialized
    return bool(vals.size and np.any(np.abs(vals.astype(np.float64)) > 32767))


def compress_payloads(boxes: Sequence[np.ndarray], keep: float, device: int = 0):
    """Batched forward path: list of Box3D -> list of serialized payload bytes.

    One wc_forward_host_units call for the whole list (all units in one launch
    set, each uploaded from its own array: no packing copy on the host, as the
    C++ mirror's compress())."""
    dims = [_box_dims(b) for b in boxes]
    units, n, _ = capi.make_units(dims)
    arrs = [np.ascontiguousarray(b, np.float32) for b in boxes]
    payload, offsets, kept = context(device).forward_host_units(arrs, units, n, keep)
    return [capi.unit_payload(payload, offsets, kept, i) for i in range(n)]


def compress(box: Sequence[np.ndarray], components: Sequence[int], keep: float, time: int,
             level: int, box_index: int, compressed_dir) -> List[CompressedWavelet]:
    """src/compressor.cpp:192-297.  box[c] is positional; components[c] (an
    AMReX header index) only names the output file.  Writes one .xz file per
    component and returns the CompressedWavelet structs."""
    comps = list(components)
    boxes = [box[c] for c in range(len(comps))]
    payloads = compress_payloads(boxes, keep)
    out = []
    for c, p in enumerate(payloads):
        cw = deserialize_compressed_wavelet(p)
        cw.need32 = _pairs_need32(np.array([v for _, v in cw.rle_encoded], np.float32))
        fname = Path(compressed_dir) / f"compressed-wavelet-{time}-{level}-{comps[c]}-{box_index}.xz"
        try:
            f = open(fname, "wb")
        except OSError:
            f = None  # a failed ofstream open silently skips the file (src/compressor.cpp:256-257)
        if f is not None:
            with f:
                f.write(lzma.compress(p, format=lzma.FORMAT_XZ, check=XZ_CHECK, preset=xz_preset()))
        out.append(cw)
    return out


def read_compressed_payload(file_path) -> bytes:
    """xz read of src/decompressor.cpp:164-220 (errors exit, as the reference does)."""
    try:
        raw = Path(file_path).read_bytes()
    except OSError as e:
        print(f"[error] Failed to open file: {file_path} ({e})", file=sys.stderr)
        sys.exit(1)
    try:
        return lzma.decompress(raw, format=lzma.FORMAT_XZ)
    except lzma.LZMAError as e:
        print(f"[error] LZMA decompression failed: {e}", file=sys.stderr)
        sys.exit(1)


def decompress_payloads(payloads: Sequence[bytes], device: int = 0) -> List[np.ndarray]:
    """Batched inverse path: serialized payloads -> Box3D arrays (one wc_inverse_host call)."""
    dims = []
    for p in payloads:
        h = np.frombuffer(p[:20], "<i4")
        dims.append((int(h[0]), int(h[1]), int(h[2])))
    units, n, extent = capi.make_units(dims)
    offsets = np.zeros(max(n, 1), np.uint64)
    cur = 4
    for i, p in enumerate(payloads):
        offsets[i] = cur
        cur += (len(p) + 4 + 7) // 8 * 8
    buf = np.zeros(cur + 8, np.uint8)
    for i, p in enumerate(payloads):
        o = int(offsets[i])
        buf[o:o + len(p)] = np.frombuffer(p, np.uint8)
    flat = context(device).inverse_host(buf, offsets, units, n, extent)
    out = []
    for i, (W, H, D) in enumerate(dims):
        o = units[i].cell_offset
        out.append(flat[o:o + W * H * D].reshape(D, H, W).copy())
    return out


def decompress(file_path, time: int = 0, level: int = 0, component: int = 0, box_idx: int = 0) -> np.ndarray:
    """src/decompressor.cpp:238-255 (only file_path is used, as in the reference)."""
    return decompress_payloads([read_compressed_payload(file_path)])[0]


def inverse_wavelet_decompose(flat, x: int, y: int, z: int) -> np.ndarray:
    """src/decompressor.cpp:79-159 on the GPU: flat coefficients -> Box3D (z, y, x)."""
    f = np.ascontiguousarray(flat, np.float32)
    if f.size != x * y * z:
        raise ValueError("flat length != x*y*z")
    units, n, extent = capi.make_units([(x, y, z)])
    return context(0).inverse_flat_host(f, units, n, extent).reshape(z, y, x)


def wavelet_decompose(box: np.ndarray) -> np.ndarray:
    """src/compressor.cpp:85-185 (static there) on the GPU: Box3D -> flat coefficients."""
    W, H, D = _box_dims(box)
    units, n, extent = capi.make_units([(W, H, D)])
    return context(0).decompose_host(np.ascontiguousarray(box, np.float32).ravel(), units, n, extent)


def calc_rmse_per_box(actual: Sequence[np.ndarray], pred: Sequence[np.ndarray],
                      num_components: int) -> List[float]:
    """src/calc-loss.cpp:12-43 on the GPU (one K7 launch for all components).
    Like the reference, every component uses actual[0]'s dimensions."""
    W, H, D = _box_dims(actual[0])
    units, n, extent = capi.make_units([(W, H, D)] * num_components)
    a = np.zeros(max(extent, 1), np.float32)
    p = np.zeros(max(extent, 1), np.float32)
    for c in range(num_components):
        o = units[c].cell_offset
        a[o:o + W * H * D] = np.ascontiguousarray(actual[c], np.float32).ravel()
        p[o:o + W * H * D] = np.ascontiguousarray(pred[c], np.float32).ravel()
    return context(0).rmse_host(a, p, units, n).tolist()


def calc_adj_loss(rmse: float, value_range: float) -> float:
    """src/calc-loss.cpp:49-51."""
    return rmse / value_range


def calc_size(path) -> float:
    """src/calc-loss.cpp:55-65: total bytes of the files under path."""
    total = 0.0
    for root, _dirs, files in os.walk(path):
        for f in files:
            total += os.path.getsize(os.path.join(root, f))
    return total
