"""AMReX plotfile reading without AMReX.

Replaces the reference's use of amrex::VisMF::Read and its Header parsing:
  read_header      src/preprocess.cpp:131-242  (plotfile Header -> names, time,
                                                geometry, ref ratios, domain, steps)
  read_level       src/preprocess.cpp:14-102   (Level_N/Cell_H + Cell_D FABs)
  preprocess_data  src/preprocess.cpp:107-307  (timesteps x levels -> boxes,
                                                locations, dimensions, min/max)

Box data comes back as float64 arrays of shape (ncomp, D, H, W) — the on-disk
FAB layout (component-major, x fastest) — so it can go to HBM unchanged and be
narrowed to float32 inside the transform kernel (the reference narrows on load,
src/preprocess.cpp:78).
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Sequence, Tuple

import numpy as np

FLT_MAX = np.float32(3.4028234663852886e38)
FLT_MIN = np.float32(1.1754943508222875e-38)  # std::numeric_limits<float>::min(): smallest positive normal

_BOX_RE = re.compile(r"\(\((-?\d+),(-?\d+),(-?\d+)\)\s*\((-?\d+),(-?\d+),(-?\d+)\)\s*\((-?\d+),(-?\d+),(-?\d+)\)\)")


@dataclass
class PlotfileHeader:
    version: str
    names: List[str]
    dim: int
    time: float
    finest_level: int
    prob_lo: List[float]
    prob_hi: List[float]
    ref_ratios: List[int]
    domains: List[Tuple[Tuple[int, int, int], Tuple[int, int, int]]]
    level_steps: List[int]
    raw_lines: List[str] = field(default_factory=list)

    @property
    def ncomp(self) -> int:
        return len(self.names)

    @property
    def domain_dims(self) -> Tuple[int, int, int]:
        """Level-0 domain size, the reference's AMReXInfo x/y/zDim (hi + 1)."""
        (_, hi) = self.domains[0]
        return hi[0] + 1, hi[1] + 1, hi[2] + 1


def read_header(plotfile_dir) -> PlotfileHeader:
    """Parse <plotfile>/Header the way src/preprocess.cpp:131-242 does."""
    lines = Path(plotfile_dir, "Header").read_text().splitlines()
    it = iter(lines)
    version = next(it).strip()
    ncomp = int(next(it))
    names = [next(it).strip() for _ in range(ncomp)]
    dim = int(next(it))
    time = float(next(it))
    finest = int(next(it))
    prob_lo = [float(v) for v in next(it).split()]
    prob_hi = [float(v) for v in next(it).split()]
    ref_line = next(it).split()
    ref_ratios = [int(v) for v in ref_line]
    domain_line = next(it)
    domains = []
    for m in _BOX_RE.finditer(domain_line):
        v = [int(x) for x in m.groups()]
        domains.append(((v[0], v[1], v[2]), (v[3], v[4], v[5])))
    steps = [int(v) for v in next(it).split()]
    return PlotfileHeader(version, names, dim, time, finest, prob_lo, prob_hi, ref_ratios, domains, steps,
                          raw_lines=lines)


@dataclass
class Fab:
    lo: Tuple[int, int, int]
    hi: Tuple[int, int, int]
    data: np.ndarray  # float64, (ncomp, D, H, W)

    @property
    def dims(self) -> Tuple[int, int, int]:
        return tuple(h - l + 1 for l, h in zip(self.lo, self.hi))


def _parse_real_descriptor(hdr: str):
    # "FAB ((8, (64 11 52 0 1 12 0 1023)),(8, (8 7 6 5 4 3 2 1)))((lo) (hi) (t)) ncomp"
    m = re.match(r"FAB \(\((\d+), \(([\d ]+)\)\),\((\d+), \(([\d ]+)\)\)\)(.*)\s(\d+)\s*$", hdr)
    if not m:
        raise ValueError(f"unrecognised FAB header: {hdr!r}")
    nbytes = int(m.group(1))
    order = [int(x) for x in m.group(4).split()]
    if nbytes != 8:
        raise ValueError("only IEEE double FABs are supported")
    if order == list(range(8, 0, -1)):
        dt = np.dtype("<f8")
    elif order == list(range(1, 9)):
        dt = np.dtype(">f8")
    else:
        raise ValueError(f"unsupported byte order {order}")
    box = _BOX_RE.search(m.group(5))
    v = [int(x) for x in box.groups()]
    return dt, (v[0], v[1], v[2]), (v[3], v[4], v[5]), int(m.group(6))


def read_level(plotfile_dir, level: int) -> List[Fab]:
    """All FABs of <plotfile>/Level_<level>/Cell (VisMF "new format", src/preprocess.cpp:36)."""
    ldir = Path(plotfile_dir, f"Level_{level}")
    lines = (ldir / "Cell_H").read_text().splitlines()
    fabs_on_disk = []
    for ln in lines:
        if ln.startswith("FabOnDisk:"):
            _, fname, off = ln.split()
            fabs_on_disk.append((fname, int(off)))
    out = []
    cache = {}
    for fname, off in fabs_on_disk:
        path = ldir / fname
        if path not in cache:
            cache[path] = np.memmap(path, dtype=np.uint8, mode="r")
        mm = cache[path]
        end = off
        while mm[end] != 0x0A:  # header line ends at '\n'
            end += 1
        hdr = bytes(mm[off:end]).decode()
        dt, lo, hi, ncomp = _parse_real_descriptor(hdr)
        W, H, D = (h - l + 1 for l, h in zip(lo, hi))
        n = ncomp * W * H * D
        raw = np.frombuffer(mm[end + 1:end + 1 + 8 * n], dtype=dt, count=n)
        out.append(Fab(lo, hi, raw.astype(np.float64).reshape(ncomp, D, H, W)))
    return out


@dataclass
class AllData:
    """src/box-structs.h:53-61.  boxes[t][lev][box] = float64 (ncomp_selected, D, H, W)."""
    boxes: list
    locations: list
    dimensions: list
    box_counts: list
    min_values: List[np.float32]
    max_values: List[np.float32]
    comp_idxs: List[int]
    headers: List[PlotfileHeader]


def preprocess_data(files: Sequence[str], components: Sequence[str], levels: Sequence[int]) -> AllData:
    """src/preprocess.cpp:107-307: components are matched in HEADER order (:152-160);
    min/max are tracked over the float32-narrowed values with the reference's
    initial values FLT_MAX / FLT_MIN (so an all-negative component reports
    max = FLT_MIN)."""
    comp_idxs: List[int] = []
    headers = []
    boxes, locs, dims, counts = [], [], [], []
    mins = [FLT_MAX] * len(components)
    maxs = [FLT_MIN] * len(components)
    for i, f in enumerate(files):
        h = read_header(f)
        headers.append(h)
        if i == 0:
            comp_idxs = [n for n, name in enumerate(h.names) if name in components]
            if len(comp_idxs) != len(components):
                raise ValueError("Some components you entered were not found in the AMReX Header")
        fb, fl, fd, fc = [], [], [], []
        for lev in levels:
            fabs = read_level(f, lev)
            lb, ll, ld = [], [], []
            for fab in fabs:
                sel = fab.data[comp_idxs]
                lb.append(sel)
                ll.append(list(fab.lo))
                ld.append(list(fab.dims))
                for c in range(len(comp_idxs)):
                    v32 = sel[c].astype(np.float32)
                    mn, mx = v32.min(), v32.max()
                    if mn < mins[c]:
                        mins[c] = mn
                    if mx > maxs[c]:
                        maxs[c] = mx
            fb.append(lb)
            fl.append(ll)
            fd.append(ld)
            fc.append(len(fabs))
        boxes.append(fb)
        locs.append(fl)
        dims.append(fd)
        counts.append(fc)
    return AllData(boxes, locs, dims, counts, mins, maxs, comp_idxs, headers)


def clean_string(filename: str) -> int:
    """src/argparse.cpp:102-125: the digits of the string as an int, -1 if none."""
    digits = "".join(ch for ch in filename if ch.isdigit())
    if not digits:
        return -1
    return int(digits)  # leading zeros dropped; all zeros -> 0


def format_files(data_dir: str, min_time: str, max_time: str) -> List[str]:
    """src/argparse.cpp:130-160: entries of data_dir whose clean_string() lies in
    [minfile, maxfile], sorted by it.  The digits are taken from the WHOLE path
    (quirk kept: digits in data_dir take part)."""
    first, last = clean_string(min_time), clean_string(max_time)
    files = [os.path.join(data_dir, e) for e in os.listdir(data_dir)]
    files = [f for f in files if first <= clean_string(f) <= last]
    return sorted(files, key=clean_string)


def format_levels(min_level: int, max_level: int) -> List[int]:
    """src/argparse.cpp:164-172."""
    return list(range(min_level, max_level + 1))


def _r17(v: float) -> str:
    return "%.17g" % v


def _box(lo, hi) -> str:
    return "((%d,%d,%d) (%d,%d,%d) (0,0,0))" % (lo[0], lo[1], lo[2], hi[0], hi[1], hi[2])


_FAB_REAL = "FAB ((8, (64 11 52 0 1 12 0 1023)),(8, (8 7 6 5 4 3 2 1)))"


def write_plotfile(path, names: Sequence[str], time: float, geomcell: Sequence[float], ref_ratio: int,
                   base_dims: Tuple[int, int, int], level_steps: Sequence[int], levels) -> None:
    """Single-rank amrex::WriteMultiLevelPlotfile output, as the C++ writer
    (csrc/host/writeplotfile.cpp) produces it.  levels[l] = list of
    (lo (x, y, z), data float64 (ncomp, D, H, W)).  Used by the tests to build
    plotfile inputs on machines without the reference's fixtures."""
    pdir = Path(path)
    nlev = len(levels)
    ncell = [[int(base_dims[k] * ref_ratio ** l) for k in range(3)] for l in range(nlev)]
    dx = [[(geomcell[3 + k] - geomcell[k]) / ncell[l][k] for k in range(3)] for l in range(nlev)]
    out = ["HyperCLaw-V1.1\n", f"{len(names)}\n"] + [f"{n}\n" for n in names]
    out += ["3\n", _r17(time) + "\n", f"{nlev - 1}\n"]
    out.append("".join(_r17(geomcell[k]) + " " for k in range(3)) + "\n")
    out.append("".join(_r17(geomcell[3 + k]) + " " for k in range(3)) + "\n")
    out.append("".join(f"{ref_ratio} " for _ in range(1, nlev)) + "\n")
    out.append("".join(_box((0, 0, 0), [n - 1 for n in ncell[l]]) + " " for l in range(nlev)) + "\n")
    out.append("".join(f"{s} " for s in level_steps[:nlev]) + "\n")
    for l in range(nlev):
        out.append("".join(_r17(d) + " " for d in dx[l]) + "\n")
    out.append("0\n0\n")
    for l, fabs in enumerate(levels):
        out.append(f"{l} {len(fabs)} {_r17(time)}\n{level_steps[l]}\n")
        for lo, data in fabs:
            D, H, W = data.shape[1:]
            for k, n in enumerate((W, H, D)):
                out.append(_r17(geomcell[k] + dx[l][k] * lo[k]) + " " + _r17(geomcell[k] + dx[l][k] * (lo[k] + n)) + "\n")
        out.append(f"Level_{l}/Cell\n")
        ldir = pdir / f"Level_{l}"
        ldir.mkdir(parents=True, exist_ok=True)
        offs, mins, maxs, boxes = [], [], [], []
        pos = 0
        with open(ldir / "Cell_D_00000", "wb") as f:
            for lo, data in fabs:
                D, H, W = data.shape[1:]
                hi = (lo[0] + W - 1, lo[1] + H - 1, lo[2] + D - 1)
                boxes.append(_box(lo, hi))
                hdr = (_FAB_REAL + _box(lo, hi) + f" {data.shape[0]}\n").encode()
                offs.append(pos)
                f.write(hdr)
                arr = np.ascontiguousarray(data, dtype="<f8")
                f.write(arr.tobytes())
                pos += len(hdr) + arr.nbytes
                mins.append([float(arr[c].min()) for c in range(arr.shape[0])])
                maxs.append([float(arr[c].max()) for c in range(arr.shape[0])])
        ncomp = len(names)
        ch = [f"1\n1\n{ncomp}\n0\n({len(fabs)} 0\n"] + [b + "\n" for b in boxes] + [f")\n{len(fabs)}\n"]
        ch += [f"FabOnDisk: Cell_D_00000 {o}\n" for o in offs]
        for mm in (mins, maxs):
            ch.append(f"\n{len(fabs)},{ncomp}\n")
            ch += ["".join("%.16e," % v for v in row) + "\n" for row in mm]
        ch.append("\n")
        (ldir / "Cell_H").write_text("".join(ch))
    (pdir / "Header").write_text("".join(out))
