"""BASELINE.json configs run on the GPU, checked against the CPU oracle.

C1 (configs[0]): the reference's own fixtures tests/plt00074 -> plt00075
    (regenerated here with the Python plotfile writer, which
    tests/test_host_io.py proves byte-identical to the reference's files, so
    nothing reads /root/reference), level 0, component temp, keep 0.999,
    -estimate through the CLI (src/modes.cpp:209-327): RMSE 0, adjusted loss 0,
    compressed size = sum of the .xz bytes / the level's raw size per component;
    then -c and -d over both fixtures, both levels and components: the
    regenerated plotfiles are the fixture files byte for byte.
C3 (configs[2]): the 4-level AMR layout x 4 components (bench_workloads.py,
    SURVEY.md §8(d)), wc_forward -> wc_inverse -> wc_rmse on one GPU through
    the C-ABI; payload bytes and reconstructions bit-exact against the oracle
    on a per-level, per-component sample, per-box RMSE within 1e-6 relative of
    calc_rmse_per_box (src/calc-loss.cpp:12-43); size-independent checks on
    every unit (headers, kept counts, RMSE of the exact reconstruction).
"""
import os
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
CLI = ROOT / "wavelet-compression_amd" / "bin" / "wavelet-compression"


def _cli(*args, env=None):
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([str(CLI), *map(str, args)], capture_output=True, text=True, timeout=600, env=e)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "[error]" not in r.stderr, r.stderr
    return r.stdout + r.stderr


@pytest.fixture
def digit_free_dir():
    # format_files takes the digits of the WHOLE path (reference quirk,
    # src/argparse.cpp:146), so the scratch root must not contain any
    import random
    import shutil
    import string
    import tempfile
    name = "wcamd_cone_" + "".join(random.choice(string.ascii_lowercase) for _ in range(10))
    p = Path(tempfile.gettempdir()) / name
    assert not re.search(r"\d", str(p))
    p.mkdir()
    yield p
    shutil.rmtree(p, ignore_errors=True)


def test_c1_estimate_on_reference_fixtures(digit_free_dir):
    from wavelet_compression_amd import plotfile as pf
    # tests/plt0007{4,5} exactly as the reference's writer test produces them
    # (src/writeplotfile.cpp:315-402; byte equality in tests/test_host_io.py)
    base = digit_free_dir
    b1 = np.full((2, 64, 32, 16), np.float32(3902.4), np.float64)
    b2 = np.full((2, 2, 4, 8), 16.0)
    lev = [((0, 0, 0), b1), ((16, 32, 64), b2)]
    for name, t, steps in (("plt00074", 0.2219392, [1200, 1500]), ("plt00075", 0.3874982, [1800, 2000])):
        pf.write_plotfile(base / "data" / name, ["temp", "pressure"], t, [0.6, 0.5, 0.4, 0.8, 0.9, 1.0], 2,
                          (256, 512, 256), steps, [lev, lev])
    out = _cli(f"datadir={base}/data/", "minfile=plt00074", "maxfile=plt00075", "minlevel=0", "maxlevel=0",
               "components=temp", "keep=0.999", f"compresseddir={base}/unused/", "-estimate")
    rmse = float(re.search(r"Predicted RMSE, temp = (\S+)", out).group(1))
    loss = float(re.search(r"Predicted Adjusted loss, temp = (\S+)", out).group(1))
    size = float(re.search(r"Predicted compressed size: (\S+)%", out).group(1))
    assert rmse == 0.0 and loss == 0.0
    # the same units compressed with -c: the .xz bytes estimate sums
    comp = base / "comp"
    _cli(f"datadir={base}/data/", "minfile=plt00074", "maxfile=plt00074", "minlevel=0", "maxlevel=0",
         "components=temp", "keep=0.999", f"compresseddir={comp}/", "-c")
    xz = sum((comp / f"compressed-wavelet-0-0-0-{b}.xz").stat().st_size for b in range(2))
    lvl = base / "data" / "plt00074" / "Level_0"
    raw = sum(f.stat().st_size for f in lvl.iterdir()) / 2 * 1
    assert raw == 262913.5  # the reference fixture's Level_0 (Cell_D_00000 + Cell_H) per component
    assert size == pytest.approx(xz / raw * 100, rel=1e-12)
    assert size == pytest.approx(0.0974, abs=0.002)  # SURVEY §6 (liblzma-version dependent)

    # -c then -d over both fixtures, both levels, both components: the boxes are
    # constant (3902.4f, 16.0), so the Haar round trip is exact and the
    # regenerated plotfiles must be the reference's own fixture files byte for
    # byte (the writer's byte identity: tests/test_host_io.py)
    import filecmp
    full = base / "full"
    _cli(f"datadir={base}/data/", "minfile=plt00074", "maxfile=plt00075", "minlevel=0", "maxlevel=1",
         "components=temp pressure", "keep=0.999", f"compresseddir={full}/", "-c")
    _cli(f"compresseddir={full}/", f"out={base}/regen/", "-d")
    for name in ("plt00074", "plt00075"):
        want = base / "data" / name
        n = 0
        for root, _, files in os.walk(want):
            for f in files:
                a = Path(root) / f
                b = base / "regen" / name / a.relative_to(want)
                assert filecmp.cmp(a, b, shallow=False), b
                n += 1
        assert n == 5  # Header, Level_{0,1}/Cell_H and Level_{0,1}/Cell_D_00000


@pytest.fixture(scope="module")
def c3_run(wc):
    import torch
    import bench_workloads as bw
    units = bw.WORKLOADS["c3"]["units"]()
    keep = float(np.float32(0.999))
    dev = torch.device("cuda", 0)
    cells, offs, extent = bw.synth_cells(torch, dev, units, "f64")
    tab, n, _ = bw.units_array(wc.capi, units, offs)
    ctx = wc.capi.Context(0)
    cap = wc.capi.payload_bound(tab, n)
    payload = torch.empty(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    regen = torch.full((extent,), float("nan"), dtype=torch.float32, device=dev)
    rmse = torch.zeros(n, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    ctx.forward(cells.data_ptr(), wc.capi.WC_F64, tab, n, keep, payload.data_ptr(), cap, offsets.data_ptr(),
                kept.data_ptr())
    ctx.inverse(payload.data_ptr(), offsets.data_ptr(), tab, n, regen.data_ptr())
    ctx.rmse(cells.data_ptr(), wc.capi.WC_F64, regen.data_ptr(), tab, n, rmse.data_ptr())
    ctx.synchronize()
    yield dict(units=units, offs=offs, cells=cells, payload=payload, offsets=offsets.cpu().numpy(),
               kept=kept.cpu().numpy(), regen=regen, rmse=rmse.cpu().numpy(), keep=keep)
    ctx.close()


def _sample(units, per_group=2, seed=3):
    rng = np.random.default_rng(seed)
    groups = {}
    for i, u in enumerate(units):
        groups.setdefault((u.lev, u.comp, (u.W, u.H, u.D)), []).append(i)
    out = []
    for key in sorted(groups):
        idx = groups[key]
        out += [idx[0]] + list(rng.choice(idx[1:], size=min(per_group - 1, len(idx) - 1), replace=False))
    return sorted(out)


def test_c3_payloads_and_reconstruction_match_oracle(c3_run, oracle):
    r = c3_run
    units = r["units"]
    sample = _sample(units)
    assert {units[i].lev for i in sample} == {0, 1, 2, 3}
    for i in sample:
        u = units[i]
        o = r["offs"][i]
        box = oracle.narrow(r["cells"][o:o + u.cells].cpu().numpy().reshape(u.D, u.H, u.W))
        want, wk = oracle.compress_payload(box, r["keep"])
        po = int(r["offsets"][i])
        got = r["payload"][po:po + 20 + 8 * int(r["kept"][i])].cpu().numpy().tobytes()
        assert got == want, (i, u)
        assert int(r["kept"][i]) == wk
        back = oracle.decompress_payload(want)
        assert r["regen"][o:o + u.cells].cpu().numpy().tobytes() == back.ravel().tobytes(), (i, u)
        ref = oracle.rmse(box, back)
        assert r["rmse"][i] == pytest.approx(ref, rel=1e-6, abs=1e-300), (i, u)


def test_c3_every_unit_size_independent(c3_run, oracle):
    """All 2304 units: headers, kept bounds, and RMSE of an exact reconstruction
    equal to the RMSE the oracle computes from the GPU's own reconstruction."""
    r = c3_run
    units = r["units"]
    pay = r["payload"].cpu().numpy()
    for i, u in enumerate(units):
        po = int(r["offsets"][i])
        hdr = np.frombuffer(pay[po:po + 20].tobytes(), "<i4")
        assert hdr.tolist() == [u.W, u.H, u.D, u.cells, int(r["kept"][i])], (i, u)
        assert 0 <= r["kept"][i] <= u.cells
    assert np.all(np.isfinite(r["rmse"])) and np.all(r["rmse"] >= 0)
    frac = r["kept"].sum() / sum(u.cells for u in units)
    assert 0.05 < frac < 0.95
    # RMSE of every 97th unit recomputed by the oracle from the GPU reconstruction
    for i in range(0, len(units), 97):
        u = units[i]
        o = r["offs"][i]
        box = oracle.narrow(r["cells"][o:o + u.cells].cpu().numpy().reshape(u.D, u.H, u.W))
        rg = r["regen"][o:o + u.cells].cpu().numpy().reshape(u.D, u.H, u.W)
        assert r["rmse"][i] == pytest.approx(oracle.rmse(box, rg), rel=1e-12, abs=1e-300), (i, u)
