"""Expected payload and reconstruction of a box TILED from a small box B.

Test infrastructure: `tests/test_tiled_model.py` pins it against the oracle on
the CPU; `tests/test_gpu_maxsize.py` uses it at the format's largest unit
sizes, where the oracle itself would take minutes per box.

The one-level Haar transform is blockwise (src/compressor.cpp:85-185: each
2x2x2 block of cells yields one coefficient in each of the 8 sub-bands), so
for a box X tiled from B (even dims, X's dims multiples of B's) the
coefficient of X at flat (I, J, K), flat = (I*H + J)*D + K (:178-181), is B's
coefficient at (m_W(I), m_H(J), m_D(K)) with
    m_N(i) = s*(n/2) + (i - s*N/2) mod (n/2),   s = [i >= N/2]
(n = B's extent on that axis).  Every copy of B's largest |c| carries its
sign, so when B's largest |c| is unique the signed max and the threshold
(:212-216) are B's; X's kept set and values are B's under the map, in X's
flat order; and X's reconstruction (src/decompressor.cpp:79-159, blockwise as
well) is B's reconstruction tiled.  B's payload, reconstruction and RMSE come
from the oracle.
"""
import numpy as np


def axis_map(N: int, n: int) -> np.ndarray:
    """m_N above: X's coefficient index on an axis -> B's."""
    assert N % 2 == 0 and n % 2 == 0 and N % n == 0, (N, n)
    h, hs = N // 2, n // 2
    i = np.arange(N, dtype=np.int64)
    s = (i >= h).astype(np.int64)
    return s * hs + (i - s * h) % hs


class TiledExpect:
    """B (shape (d, h, w), float32 = the narrowed cells) at `keep`."""

    def __init__(self, O, b32: np.ndarray, keep: float):
        assert b32.dtype == np.float32 and all(x % 2 == 0 for x in b32.shape)
        self.d, self.h, self.w = b32.shape
        flat = O.wavelet_decompose(b32)
        mags = np.abs(flat)
        # the precondition above: B's largest |c| is unique
        assert int((mags == mags.max()).sum()) == 1
        payload, _ = O.compress_payload(b32, keep)
        (_, _, _), nc, runs, vals = O.parse_payload(payload)
        self.payload = payload
        self.flat_kept = O.rle_decode(runs, vals, nc)  # kept values, 0 elsewhere
        pos = np.cumsum(runs.astype(np.int64) + 1) - 1
        self.mask = np.zeros(nc, bool)
        self.mask[pos] = True
        self.regen = O.decompress_payload(payload)  # (d, h, w)
        self.rmse = O.rmse(b32, self.regen)
        self.kept = int(pos.size)

    def tiled(self, torch, box: np.ndarray, dev, W: int, H: int, D: int):
        """`box` (B's cells in any dtype) tiled to X's (D, H, W), flat, on dev."""
        t = torch.from_numpy(np.ascontiguousarray(box)).to(dev)
        return t.repeat(D // self.d, H // self.h, W // self.w).reshape(-1)

    def pair_slabs(self, torch, dev, W: int, H: int, D: int, slab: int = 64):
        """X's (run, value-bits) pairs as int32 (k, 2) tensors, one per slab of
        `slab` x-rows I (flat order is I-major), in order."""
        iI, iJ, iK = (torch.from_numpy(axis_map(N, n)).to(dev)
                      for N, n in ((W, self.w), (H, self.h), (D, self.d)))
        mask3 = torch.from_numpy(self.mask.reshape(self.w, self.h, self.d)).to(dev)
        vals = torch.from_numpy(self.flat_kept).to(dev)
        mJK = mask3.index_select(1, iJ).index_select(2, iK)  # (w, H, D)
        HD = H * D
        last = -1
        for I0 in range(0, W, slab):
            I1 = min(W, I0 + slab)
            m = mJK.index_select(0, iI[I0:I1]).reshape(-1)
            pos = torch.nonzero(m).reshape(-1)
            del m
            if pos.numel() == 0:
                continue
            I = pos // HD
            r = pos - I * HD
            J = r // D
            K = r - J * D
            sidx = (iI[I0 + I] * self.h + iJ[J]) * self.d + iK[K]
            pos += I0 * HD
            runs = torch.diff(pos, prepend=pos.new_tensor([last])) - 1
            last = int(pos[-1])
            yield torch.stack([runs.to(torch.int32), vals[sidx].view(torch.int32)], dim=1)

    def regen_slabs(self, torch, dev, W: int, H: int, D: int):
        """X's reconstruction as (d, H, W) slabs of z-planes, in order."""
        t = torch.from_numpy(self.regen).to(dev).repeat(1, H // self.h, W // self.w)
        for _ in range(D // self.d):
            yield t
