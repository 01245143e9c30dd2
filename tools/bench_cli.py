"""End-to-end timing of the wavelet-compression command line (-c, -d, -estimate)
on a synthetic AMR run, with the reference-faithful CPU rate passed in (bench.py's cpu_baseline measures it).

Layout (scaled by --scale): level 0 = 64 boxes of 64^3,
level 1 = 96 x 64^3, level 2 = 128 x 32^3, level 3 = 256 x 16^3 + 32 x (48x32x16),
NCOMP components in the plotfile, all compressed, keep 0.999, fp64 FABs.
Reported: wall seconds per mode, input GB/s of -c, units/s, and -c's speedup
over --cpu-cells-per-s (the reference's per-unit compress() work incl. xz
preset 6, as bench.py's cpu_baseline times it) when given.

-c is also run with each of --fast-presets (the optional faster xz preset,
`xzpreset=N`): time, .xz bytes, and that -d regenerates identical plotfiles.

usage: python tools/bench_cli.py [--scale 1.0] [--ncomp 4] [--out profiles/r03/cli_e2e.json]
"""
from __future__ import annotations

import argparse
import json
import lzma
import os
import random
import shutil
import string
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
CLI = ROOT / "wavelet-compression_amd" / "bin" / "wavelet-compression"


def layout(scale: float):
    def n(k):
        return max(1, int(round(k * scale)))
    return [
        [(64, 64, 64)] * n(64),
        [(64, 64, 64)] * n(96),
        [(32, 32, 32)] * n(128),
        [(16, 16, 16)] * n(256) + [(48, 32, 16)] * n(32),
    ]


def place(boxes):
    """Non-overlapping lo corners on a simple x-major grid."""
    out, x, y, z, row_h = [], 0, 0, 0, 0
    for (W, H, D) in boxes:
        out.append(((x, y, z), (W, H, D)))
        x += W
        row_h = max(row_h, H)
        if x >= 1024:
            x, y = 0, y + row_h
            row_h = 0
    return out


def cli_devices() -> int:
    """The GPUs the CLI spreads a run over (host/modes.cpp run_devices): every
    visible device unless WCAMD_DEVICES / WCAMD_DEVICE pick them."""
    v, one = os.environ.get("WCAMD_DEVICES", ""), os.environ.get("WCAMD_DEVICE", "")
    if not v and one:
        return 1
    if v and v != "all":
        return len([x for x in v.split(",") if x])
    import torch  # counting devices does not initialise the GPU in this process
    return torch.cuda.device_count()


def digit_free_dir() -> Path:
    p = Path(tempfile.gettempdir()) / ("wcamd_etoe_" + "".join(random.choice(string.ascii_lowercase) for _ in range(8)))
    assert not any(ch.isdigit() for ch in str(p)), p  # format_files reads the digits of the WHOLE path
    p.mkdir()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--ncomp", type=int, default=4)
    ap.add_argument("--keep", type=float, default=0.999)
    ap.add_argument("--cpu-cells-per-s", type=float, default=None,
                    help="the reference-faithful compress() rate (cells/s incl. xz preset 6) to compare -c with: "
                         "bench.py measures it in its cpu_baseline leg (this tool runs no CPU restatement)")
    ap.add_argument("--fast-presets", default="0,1", help="xzpreset= values timed beside the default 6")
    ap.add_argument("--out", default=str(ROOT / "profiles" / "r03" / "cli_e2e.json"))
    args = ap.parse_args()
    import wcamd  # noqa: F401  (registers the package as wavelet_compression_amd)
    from wavelet_compression_amd import plotfile as pf

    def field(seed, lo, W, H, D):
        """SURVEY.md §8(d) field on a box at global corner lo, (D, H, W) fp64."""
        z, y, x = np.meshgrid(np.arange(D), np.arange(H), np.arange(W), indexing="ij")
        g = np.random.default_rng(seed).standard_normal((D, H, W))
        return (300.0 + 50.0 * np.sin(0.1 * (lo[0] + x)) * np.cos(0.07 * (lo[1] + y)) + 0.01 * (lo[2] + z)
                + 0.05 * g)

    names = [f"var_{chr(97 + i)}" for i in range(args.ncomp)]
    base = digit_free_dir()
    try:
        t0 = time.perf_counter()
        levels = []
        ncells = 0
        for l, boxes in enumerate(layout(args.scale)):
            fabs = []
            for b, (lo, (W, H, D)) in enumerate(place(boxes)):
                comps = [field((l * 100003 + b) * 16 + c, lo, W, H, D) + 100.0 * c for c in range(args.ncomp)]
                fabs.append((lo, np.stack(comps)))
                ncells += W * H * D * args.ncomp
            levels.append(fabs)
        pf.write_plotfile(base / "data" / "plt00100", names, 1.0, [0, 0, 0, 1, 1, 1], 2, (1024, 1024, 1024),
                          [10, 20, 30, 40], levels)
        t_gen = time.perf_counter() - t0
        comp = " ".join(names)
        common = [f"datadir={base}/data/", "minfile=plt00100", "maxfile=plt00100", "minlevel=0",
                  f"maxlevel={len(levels) - 1}", f"components={comp}", f"keep={args.keep}"]

        logs = {}

        def run(argv):
            t = time.perf_counter()
            r = subprocess.run([str(CLI), *argv], capture_output=True, text=True, timeout=1800)
            dt = time.perf_counter() - t
            out = r.stdout + r.stderr
            logs[argv[-1]] = out[-1500:]
            if r.returncode != 0 or "[error]" in out:
                raise SystemExit(out)
            return dt, out

        t_c, _ = run(common + [f"compresseddir={base}/comp/", "-c"])
        xz_bytes = sum(f.stat().st_size for f in (base / "comp").glob("*.xz"))
        if xz_bytes == 0:
            raise SystemExit("no .xz files written:\n" + logs["-c"])
        t_d, _ = run([f"compresseddir={base}/comp/", f"out={base}/regen/", "-d"])
        # the optional faster xz presets: same payloads, other .xz streams
        fast = {}
        for pr in args.fast_presets.split(","):
            d = base / f"comp_p{pr}"
            t_f, _ = run(common + [f"compresseddir={d}/", f"xzpreset={pr}", "-c"])
            nb = sum(f.stat().st_size for f in d.glob("*.xz"))
            same = all(lzma.decompress(f.read_bytes()) == lzma.decompress((d / f.name).read_bytes())
                       for f in sorted((base / "comp").glob("*.xz"))[::97])
            t_fd, _ = run([f"compresseddir={d}/", f"out={base}/regen_p{pr}/", "-d"])
            regen_same = all(
                f.read_bytes() == (base / f"regen_p{pr}" / f.relative_to(base / "regen")).read_bytes()
                for f in (base / "regen").rglob("*") if f.is_file())
            fast[pr] = {"compress_s": t_f, "compress_cells_per_s": ncells / t_f, "xz_bytes": nb,
                        "size_vs_preset6": nb / xz_bytes, "decompress_s": t_fd,
                        "payloads_equal_preset6_sample": bool(same), "regen_plotfiles_identical": bool(regen_same)}
            shutil.rmtree(d, ignore_errors=True)
            shutil.rmtree(base / f"regen_p{pr}", ignore_errors=True)
        t_e, est = run([*common[:3], "minlevel=0", "maxlevel=0", f"components={comp}", f"keep={args.keep}",
                        f"compresseddir={base}/x/", "-estimate"])
        nunits = sum(len(f) for f in levels) * args.ncomp

        res = {
            "workload": f"C3-like synthetic plotfile x{args.scale}: 4 levels, {args.ncomp} comps, {nunits} units, "
                        f"{ncells} cells fp64 ({ncells * 8 / 1e9:.2f} GB), keep={args.keep}",
            "compress_s": t_c, "decompress_s": t_d, "estimate_s": t_e,
            "compress_input_GBps": ncells * 8 / t_c / 1e9,
            "compress_cells_per_s": ncells / t_c,
            "decompress_cells_per_s": ncells / t_d,
            "xz_bytes": xz_bytes, "compressed_fraction": xz_bytes / (ncells * 8),
            "xz_preset": 6, "fast_xz_presets": fast,
            "gpu_devices": cli_devices(),
            "host_threads": int(os.environ.get("WCAMD_THREADS", os.environ.get("OMP_NUM_THREADS", os.cpu_count()))),
            "cpu_compress_cells_per_s": args.cpu_cells_per_s,
            "speedup_vs_cpu_compress": (ncells / t_c) / args.cpu_cells_per_s if args.cpu_cells_per_s else None,
            "generate_s": t_gen,
            "estimate_output": [ln for ln in est.splitlines() if "Predicted" in ln],
            "cli_logs": logs,
        }
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(res, indent=1) + "\n")
        print(json.dumps(res))
    finally:
        shutil.rmtree(base, ignore_errors=True)


if __name__ == "__main__":
    main()
