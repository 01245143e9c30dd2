"""End-to-end command line (-c / -d / -estimate, src/modes.cpp) on the GPU.

Inputs are synthetic AMReX plotfiles written by the Python writer (itself
byte-identical to the reference's fixture, tests/test_host_io.py), so nothing
here reads /root/reference.  Checks, per unit: the .xz stream decodes to the
oracle's payload bytes; the regenerated plotfiles equal, byte for byte, the
plotfiles of the oracle's reconstruction; estimate's RMSE / adjusted loss /
size match the oracle's."""
import lzma
import os
import random
import re
import shutil
import string
import subprocess
import tempfile
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
CLI = ROOT / "wavelet-compression_amd" / "bin" / "wavelet-compression"
NAMES = ["density", "temp", "pressure"]
COMPS = ["temp", "pressure"]          # header order -> comp_idxs [1, 2]
IDX = [1, 2]
KEEP = 0.999
GEOM = [0.0, -1.0, 0.5, 1.0, 1.0, 2.5]
LEVELS = [
    [((0, 0, 0), (32, 32, 32)), ((32, 0, 0), (16, 8, 24)), ((0, 32, 0), (7, 5, 3))],
    [((0, 0, 0), (64, 64, 16)), ((64, 0, 0), (6, 10, 14))],
]
TIMES = {"plt00010": 1.25, "plt00011": 1.5, "plt00012": 1.75}


def digit_free_dir() -> Path:
    # format_files takes the digits of the WHOLE path (reference quirk), so the
    # scratch root must not contain any
    name = "wcamd_cli_" + "".join(random.choice(string.ascii_lowercase) for _ in range(10))
    p = Path(tempfile.gettempdir()) / name
    assert not re.search(r"\d", str(p))
    p.mkdir()
    return p


@pytest.fixture(scope="module")
def run(oracle):
    from wavelet_compression_amd import plotfile as pf
    base = digit_free_dir()
    data = {}
    for ti, (name, time) in enumerate(TIMES.items()):
        levels = []
        for l, boxes in enumerate(LEVELS):
            fabs = []
            for b, (lo, (W, H, D)) in enumerate(boxes):
                comps = [oracle.synth_box_f64(oracle.unit_seed(ti, l, b, c), lo, W, H, D, sigma=0.05) * (1 + c)
                         for c in range(len(NAMES))]
                arr = np.stack(comps)  # (ncomp, D, H, W)
                fabs.append((lo, arr))
                data[(name, l, b)] = arr
            levels.append(fabs)
        pf.write_plotfile(base / "data" / name, NAMES, time, GEOM, 2, (128, 64, 64), [100 + ti, 200 + ti], levels)
    yield base, data
    shutil.rmtree(base, ignore_errors=True)


def cli(*args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([str(CLI), *map(str, args)], capture_output=True, text=True, timeout=600, env=e)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[error]" not in r.stderr, r.stderr
    return r.stdout


def expected_payload(oracle, arr, c):
    return oracle.compress_payload(oracle.narrow(arr[IDX[c]]), float(np.float32(KEEP)))[0]


@pytest.fixture(scope="module")
def compressed(run, oracle):
    base, data = run
    out = base / "comp"
    # small chunks: several GPU batches + overlapped xz stages
    cli(f"datadir={base}/data/", "minfile=plt00010", "maxfile=plt00011", "minlevel=0", "maxlevel=1",
        "components=temp pressure", f"keep={KEEP}", f"compresseddir={out}/", "-c",
        env={"WCAMD_CHUNK_CELLS": "60000", "WCAMD_THREADS": "4"})
    return out


def test_compress_writes_reference_payloads(run, compressed, oracle):
    base, data = run
    for t, name in enumerate(["plt00010", "plt00011"]):
        for l, boxes in enumerate(LEVELS):
            for b in range(len(boxes)):
                for c, comp in enumerate(IDX):
                    f = compressed / f"compressed-wavelet-{t}-{l}-{comp}-{b}.xz"
                    got = lzma.decompress(f.read_bytes(), format=lzma.FORMAT_XZ)
                    assert got == expected_payload(oracle, data[(name, l, b)], c), f
    assert not list(compressed.glob("compressed-wavelet-2-*"))  # plt00012 is outside [minfile, maxfile]


def test_compress_side_files(compressed):
    counts = np.fromfile(compressed / "boxcounts.raw", np.float32)
    assert counts.tolist() == [3, 2, 3, 2]
    locs = np.fromfile(compressed / "locations.raw", np.float32).reshape(-1, 3)
    dims = np.fromfile(compressed / "dimensions.raw", np.float32).reshape(-1, 3)
    flat = [b for _ in range(2) for boxes in LEVELS for b in boxes]
    assert locs.tolist() == [list(lo) for lo, _ in flat]
    assert dims.tolist() == [list(d) for _, d in flat]


def test_decompress_regenerates_plotfiles(run, compressed, oracle, tmp_path):
    from wavelet_compression_amd import plotfile as pf
    import filecmp
    base, data = run
    out = base / "regen"
    cli(f"compresseddir={compressed}/", f"out={out}/", "-d", env={"WCAMD_THREADS": "3"})
    for t, name in enumerate(["plt00010", "plt00011"]):
        levels = []
        for l, boxes in enumerate(LEVELS):
            fabs = []
            for b, (lo, _) in enumerate(boxes):
                recon = [oracle.decompress_payload(expected_payload(oracle, data[(name, l, b)], c)) for c in range(2)]
                fabs.append((lo, np.stack(recon).astype(np.float64)))
            levels.append(fabs)
        want = tmp_path / name
        pf.write_plotfile(want, COMPS, TIMES[name], GEOM, 2, (128, 64, 64), [100 + t, 200 + t], levels)
        for root, _, files in os.walk(want):
            for f in files:
                a = Path(root) / f
                b = out / name / a.relative_to(want)
                assert filecmp.cmp(a, b, shallow=False), b


def test_estimate_matches_oracle(run, compressed, oracle):
    base, data = run
    out = cli(f"datadir={base}/data/", "minfile=plt00010", "maxfile=plt00012", "minlevel=1", "maxlevel=1",
              "components=temp pressure", f"keep={KEEP}", f"compresseddir={base}/unused/", "-estimate")
    got = {k: float(v) for k, v in re.findall(r"Predicted RMSE, (\w+) = (\S+)", out)}
    loss = {k: float(v) for k, v in re.findall(r"Predicted Adjusted loss, (\w+) = (\S+)", out)}
    size = float(re.search(r"Predicted compressed size: (\S+)%", out).group(1))
    xz_bytes = 0
    for c, comp in enumerate(COMPS):
        rm, lo, hi = [], np.float32(3.4028234663852886e38), np.float32(1.1754943508222875e-38)
        for b in range(len(LEVELS[1])):
            arr = data[("plt00010", 1, b)]
            a32 = oracle.narrow(arr[IDX[c]])
            p = expected_payload(oracle, arr, c)
            rm.append(oracle.rmse(a32, oracle.decompress_payload(p)))
            lo, hi = min(lo, a32.min()), max(hi, a32.max())
            xz_bytes += (compressed / f"compressed-wavelet-0-1-{IDX[c]}-{b}.xz").stat().st_size
        mean = sum(rm) / len(rm)
        assert got[comp] == pytest.approx(mean, rel=1e-12, abs=1e-300)
        assert loss[comp] == pytest.approx(mean / (float(hi) - float(lo)), rel=1e-12, abs=1e-300)
    lvl = base / "data" / "plt00010" / "Level_1"
    raw = sum(f.stat().st_size for f in lvl.iterdir()) / len(NAMES) * len(COMPS)
    assert size == pytest.approx(xz_bytes / raw * 100, rel=1e-12)


def test_multi_device_workers_write_identical_files(run, compressed, tmp_path):
    """Chunks (and -d timesteps) spread over one host thread + context per
    device: every visible device by default, WCAMD_DEVICES picks them ("0,0"
    runs the multi-device path on a one-GPU box), WCAMD_DEVICE pins one."""
    import filecmp
    base, _ = run
    out = base / "comp_md"
    cli(f"datadir={base}/data/", "minfile=plt00010", "maxfile=plt00011", "minlevel=0", "maxlevel=1",
        "components=temp pressure", f"keep={KEEP}", f"compresseddir={out}/", "-c",
        env={"WCAMD_CHUNK_CELLS": "60000", "WCAMD_DEVICES": "0,0", "WCAMD_THREADS": "4"})
    names = sorted(p.name for p in compressed.iterdir())
    assert names == sorted(p.name for p in out.iterdir())
    for n in names:
        assert filecmp.cmp(compressed / n, out / n, shallow=False), n
    r1, r2 = base / "regen_md1", base / "regen_md2"
    cli(f"compresseddir={compressed}/", f"out={r1}/", "-d", env={"WCAMD_DEVICE": "0"})
    cli(f"compresseddir={out}/", f"out={r2}/", "-d", env={"WCAMD_DEVICES": "0,0"})
    for root, _, files in os.walk(r1):
        for f in files:
            a = Path(root) / f
            assert filecmp.cmp(a, r2 / a.relative_to(r1), shallow=False), a
    # -estimate over two device workers (chunks of one box each, in any order):
    # the same RMSE / adjusted loss / size lines as one device (the per-box
    # RMSEs are averaged in iterator order whatever chunk finishes first)
    args = (f"datadir={base}/data/", "minfile=plt00010", "maxfile=plt00012", "minlevel=0", "maxlevel=0",
            "components=temp pressure", f"keep={KEEP}", f"compresseddir={base}/unused/", "-estimate")
    want = re.findall(r"Predicted .*", cli(*args, env={"WCAMD_DEVICE": "0"}))
    got = re.findall(r"Predicted .*", cli(*args, env={"WCAMD_CHUNK_CELLS": "20000", "WCAMD_DEVICES": "0,0",
                                                     "WCAMD_THREADS": "4"}))
    assert len(want) == 5 and got == want
    # no device variable: every visible device (this box's one GPU), same lines
    assert re.findall(r"Predicted .*", cli(*args, env={"WCAMD_CHUNK_CELLS": "20000"})) == want


def test_fast_xz_preset_round_trip(run, compressed, tmp_path):
    """`xzpreset=0` (not a reference parameter): every .xz
    decodes to the same payload as the default preset-6 file, the files differ
    (another filter preset), and -d regenerates the same plotfiles."""
    import filecmp
    base, _ = run
    out = base / "comp_p0"
    cli(f"datadir={base}/data/", "minfile=plt00010", "maxfile=plt00011", "minlevel=0", "maxlevel=1",
        "components=temp pressure", f"keep={KEEP}", f"compresseddir={out}/", "xzpreset=0", "-c",
        env={"WCAMD_CHUNK_CELLS": "60000", "WCAMD_THREADS": "4"})
    xz6 = sorted(compressed.glob("*.xz"))
    assert xz6 and sorted(p.name for p in out.glob("*.xz")) == [p.name for p in xz6]
    differ = 0
    for f in xz6:
        a, b = f.read_bytes(), (out / f.name).read_bytes()
        assert lzma.decompress(a) == lzma.decompress(b), f.name
        differ += a != b
    assert differ > 0
    r6, r0 = base / "regen_p6", base / "regen_p0"
    cli(f"compresseddir={compressed}/", f"out={r6}/", "-d")
    cli(f"compresseddir={out}/", f"out={r0}/", "-d")
    for root, _, files in os.walk(r6):
        for f in files:
            a = Path(root) / f
            assert filecmp.cmp(a, r0 / a.relative_to(r6), shallow=False), a
