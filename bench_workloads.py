"""Synthetic workloads of BASELINE.json's configs, shared by
bench.py and the GPU tests.  Benchmark/test infrastructure, not product code.

A workload is a list of units, one per (timestep, level, box, component) in
the reference's iteration order (src/iterator.h:25-33 over t, level, box;
components inside compress(), src/compressor.cpp:203): each unit is one
Box3D component, W x H x D cells at a global index offset `lo`.

Field (generalised per component c and timestep t):
    v = mean_c + amp_c * sin(0.1 * (gx + 3t)) * cos(0.07 * gy) + 0.01 * gz + 0.05 * N(0, 1)
with g = lo + local index.  Component 0 is exactly the survey's field
(mean 300, amplitude 50).  Components with mean 0 have a box average whose
sign varies from box to box, so some boxes' signed max is negative (the
reference then keeps every coefficient, src/compressor.cpp:212-226).  The
noise is a counter-based hash of (unit id, cell index), so a unit's cells do
not depend on how units are sharded over ranks.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Sequence, Tuple

COMP_MEAN = (300.0, 1000.0, 5.0, 0.0, 300.0, 1.0, 50.0, 0.0)
COMP_AMP = (50.0, 120.0, 2.0, 40.0, 80.0, 0.5, 10.0, 3.0)
SIGMA = 0.05


@dataclass(frozen=True)
class Unit:
    t: int
    lev: int
    box: int
    comp: int
    W: int
    H: int
    D: int
    lo: Tuple[int, int, int]
    gid: int  # global unit id (noise stream)

    @property
    def cells(self) -> int:
        return self.W * self.H * self.D


def _grid_boxes(n, dims, per_row, per_plane, z0=0):
    W, H, D = dims
    return [((i % per_row) * W, ((i // per_row) % per_plane) * H, (i // (per_row * per_plane)) * D + z0)
            for i in range(n)]


def amr_levels():
    """The 4-level AMR layout of C3/C4:
    L0 64 x 64^3, L1 96 x 64^3, L2 128 x 32^3, L3 256 x 16^3 + 32 x (48 x 32 x 16).
    Returns [(level, [(dims, lo), ...])]."""
    levels = []
    levels.append((0, [((64, 64, 64), lo) for lo in _grid_boxes(64, (64, 64, 64), 4, 4)]))
    levels.append((1, [((64, 64, 64), lo) for lo in _grid_boxes(96, (64, 64, 64), 6, 4)]))
    levels.append((2, [((32, 32, 32), lo) for lo in _grid_boxes(128, (32, 32, 32), 8, 4)]))
    l3 = [((16, 16, 16), lo) for lo in _grid_boxes(256, (16, 16, 16), 8, 8)]
    l3 += [((48, 32, 16), lo) for lo in _grid_boxes(32, (48, 32, 16), 4, 4, z0=256)]
    levels.append((3, l3))
    return levels


def amr_units(timesteps: int, ncomp: int) -> List[Unit]:
    out = []
    for t in range(timesteps):
        for lev, boxes in amr_levels():
            for b, ((W, H, D), lo) in enumerate(boxes):
                for c in range(ncomp):
                    out.append(Unit(t, lev, b, c, W, H, D, lo, len(out)))
    return out


def cube_units(nboxes: int, dim: int) -> List[Unit]:
    """nboxes single-level dim^3 boxes of component 0 on a 16 x 8 x ... grid."""
    return [Unit(0, 0, b, 0, dim, dim, dim,
                 (dim * (b % 16), dim * ((b // 16) % 8), dim * (b // 128)), b) for b in range(nboxes)]


WORKLOADS = {
    # BASELINE.json configs[1..4]
    "c2": dict(units=lambda: cube_units(1024, 64), dtype="f64", keep=0.999, per_gpu=True,
               desc="1024 x 64^3 fp64 boxes per GPU, 1 component, keep 0.999"),
    "c3": dict(units=lambda: amr_units(1, 4), dtype="f64", keep=0.999, per_gpu=False,
               desc="4-level AMR (L0 64x64^3, L1 96x64^3, L2 128x32^3, L3 256x16^3 + 32x48x32x16), "
                    "4 components, keep 0.999, fwd + inv + RMSE"),
    "c4": dict(units=lambda: amr_units(10, 8), dtype="f64", keep=0.999, per_gpu=False,
               desc="10 timesteps x the C3 4-level layout x 8 components, keep 0.999, box-sharded"),
    "c5": dict(units=lambda: cube_units(512, 128), dtype="f32", keep=0.9999, per_gpu=False,
               desc="512 x 128^3 fp32 boxes in total, keep 0.9999, box-sharded"),
    # the drop-in compress() input type: Box3D holds fp32 cells (reference src/box-structs.h:7),
    # so the reference's own hot call (src/compressor.cpp:192) runs the fp32 forward on C2's shape
    "f32_64": dict(units=lambda: cube_units(1024, 64), dtype="f32", keep=0.999, per_gpu=True,
                   desc="1024 x 64^3 fp32 boxes per GPU (Box3D fp32, the drop-in compress() input), keep 0.999"),
}


def layout(units: Sequence[Unit], align: int = 4):
    """Cell offsets (each rounded up to `align` elements) and the extent."""
    offs, cur = [], 0
    for u in units:
        cur = (cur + align - 1) // align * align
        offs.append(cur)
        cur += u.cells
    return offs, cur


_M64 = (1 << 64) - 1


def _as_i64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def _mix64(torch, z):
    """splitmix64 finaliser on int64 tensors (wrapping arithmetic, logical shifts)."""
    def srl(x, k):
        return (x >> k) & ((1 << (64 - k)) - 1)
    z = (z ^ srl(z, 30)) * _as_i64(0xBF58476D1CE4E5B9)
    z = (z ^ srl(z, 27)) * _as_i64(0x94D049BB133111EB)
    return z ^ srl(z, 31)


def synth_cells(torch, dev, units: Sequence[Unit], dtype: str, offsets=None, chunk_cells: int = 1 << 25):
    """Generate every unit's cells on `dev` into one flat buffer (fp64 or fp32)
    at `offsets` (default: layout(units)).  Returns (buffer, offsets, extent)."""
    if offsets is None:
        offsets, extent = layout(units)
    else:
        extent = max((o + u.cells for o, u in zip(offsets, units)), default=0)
    td = torch.float64 if dtype == "f64" else torch.float32
    out = torch.zeros(max(extent, 1), dtype=td, device=dev)
    groups = {}
    for i, u in enumerate(units):
        groups.setdefault((u.W, u.H, u.D), []).append(i)
    two_pi = 6.283185307179586
    for (W, H, D), idx in groups.items():
        per = W * H * D
        step = max(1, chunk_cells // max(per, 1))
        z = torch.arange(D, device=dev, dtype=torch.float64).view(1, D, 1, 1)
        y = torch.arange(H, device=dev, dtype=torch.float64).view(1, 1, H, 1)
        x = torch.arange(W, device=dev, dtype=torch.float64).view(1, 1, 1, W)
        cell = torch.arange(per, device=dev, dtype=torch.int64).view(1, per)
        for s in range(0, len(idx), step):
            sel = [units[i] for i in idx[s:s + step]]
            B = len(sel)
            f = lambda vals: torch.tensor(vals, device=dev, dtype=torch.float64).view(B, 1, 1, 1)
            gx = x + f([u.lo[0] + 3 * u.t for u in sel])
            gy = y + f([u.lo[1] for u in sel])
            gz = z + f([u.lo[2] for u in sel])
            mean = f([COMP_MEAN[u.comp % len(COMP_MEAN)] for u in sel])
            amp = f([COMP_AMP[u.comp % len(COMP_AMP)] for u in sel])
            v = mean + amp * torch.sin(0.1 * gx) * torch.cos(0.07 * gy) + 0.01 * gz
            gid = torch.tensor([u.gid for u in sel], device=dev, dtype=torch.int64).view(B, 1)
            key = (gid << 32) | cell
            h1 = _mix64(torch, key * 2 + _as_i64(0x9E3779B97F4A7C15))
            h2 = _mix64(torch, key * 2 + 1 + _as_i64(0x9E3779B97F4A7C15))
            u1 = (((h1 >> 11) & ((1 << 53) - 1)).to(torch.float64) + 1.0) * (1.0 / 9007199254740992.0)
            u2 = ((h2 >> 11) & ((1 << 53) - 1)).to(torch.float64) * (1.0 / 9007199254740992.0)
            g = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(two_pi * u2)
            v = (v.reshape(B, per) + SIGMA * g).to(td)
            for j, i in enumerate(idx[s:s + step]):
                o = offsets[i]
                out[o:o + per] = v[j]
    return out, offsets, extent


def units_array(capi, units: Sequence[Unit], offsets):
    """The C-ABI unit table (wc_unit) for these units at these cell offsets."""
    return capi.make_units([(u.W, u.H, u.D) for u in units], offsets=offsets)
