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
    SURVEY.md §8(d)), 2304 units on one GPU through the C-ABI, in the three
    round-trip forms: wc_forward_rows + wc_inverse_rows (what bench.py's c3
    leg times), wc_forward + wc_inverse_rmse, wc_forward + wc_inverse +
    wc_rmse.  EVERY unit's payload bytes, kept count and reconstruction
    bit-exact against the oracle, its RMSE within 1e-12 of calc_rmse_per_box
    (src/calc-loss.cpp:12-43); every unit's row index against the numpy
    restatement; the three forms identical.
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


def _threads():
    return max(1, min(16, os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


@pytest.fixture(scope="module")
def c3_run(wc):
    """The C3 batch through the two paths bench.py's c3 leg times and the
    -estimate round trip: wc_forward_rows + wc_inverse_rows (the forward's row
    index, fused RMSE) and wc_forward + wc_inverse_rmse (the row index from the
    payloads); plus wc_inverse + wc_rmse, the separate calls."""
    import torch
    import bench_workloads as bw
    units = bw.WORKLOADS["c3"]["units"]()
    keep = float(np.float32(0.999))
    dev = torch.device("cuda", 0)
    cells, offs, extent = bw.synth_cells(torch, dev, units, "f64")
    tab, n, _ = bw.units_array(wc.capi, units, offs)
    ctx = wc.capi.Context(0)
    cap = wc.capi.payload_bound(tab, n)
    rb = wc.capi.rowindex_bytes(tab, n)
    F64 = wc.capi.WC_F64
    out = {}
    for path in ("rows", "fused", "separate"):
        payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
        offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
        kept = torch.zeros(n, dtype=torch.int32, device=dev)
        regen = torch.full((extent,), float("nan"), dtype=torch.float32, device=dev)
        rmse = torch.zeros(n, dtype=torch.float64, device=dev)
        rowinfo = torch.zeros(rb // 4, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        if path == "rows":
            ctx.forward_rows(cells.data_ptr(), F64, tab, n, keep, payload.data_ptr(), cap, offsets.data_ptr(),
                             kept.data_ptr(), rowinfo.data_ptr(), rb)
            ctx.inverse_rows(payload.data_ptr(), offsets.data_ptr(), tab, n, rowinfo.data_ptr(), regen.data_ptr(),
                             cells.data_ptr(), F64, rmse.data_ptr())
        else:
            ctx.forward(cells.data_ptr(), F64, tab, n, keep, payload.data_ptr(), cap, offsets.data_ptr(),
                        kept.data_ptr())
            if path == "fused":
                ctx.inverse_rmse(payload.data_ptr(), offsets.data_ptr(), tab, n, cells.data_ptr(), F64,
                                 regen.data_ptr(), rmse.data_ptr())
            else:
                ctx.inverse(payload.data_ptr(), offsets.data_ptr(), tab, n, regen.data_ptr())
                ctx.rmse(cells.data_ptr(), F64, regen.data_ptr(), tab, n, rmse.data_ptr())
        ctx.synchronize()
        out[path] = dict(payload=payload.cpu().numpy(), offsets=offsets.cpu().numpy(), kept=kept.cpu().numpy(),
                         regen=regen.cpu().numpy(), rmse=rmse.cpu().numpy(),
                         rowinfo=rowinfo.cpu().numpy().view(np.uint32).reshape(-1, 2))
        del payload, regen, rowinfo
    r = dict(units=units, offs=offs, cells=cells.cpu().numpy(), keep=keep, **out)
    ctx.close()
    del cells
    torch.cuda.empty_cache()
    yield r


def _box(r, i):
    u = r["units"][i]
    o = r["offs"][i]
    return r["cells"][o:o + u.cells].reshape(u.D, u.H, u.W)


def _payload(p, i):
    po = int(p["offsets"][i])
    return p["payload"][po:po + 20 + 8 * int(p["kept"][i])].tobytes()


def test_c3_every_unit_matches_oracle(c3_run, oracle):
    """All 2304 C3 units through wc_forward_rows + wc_inverse_rows (the c3
    leg of bench.py and -estimate): every payload and kept count equal the
    oracle's compress() minus xz, every reconstruction its decompress() bit for
    bit, every RMSE within 1e-12 of calc_rmse_per_box (src/calc-loss.cpp:12-43)."""
    from concurrent.futures import ThreadPoolExecutor
    r = c3_run
    p = r["rows"]
    units = r["units"]
    assert {u.lev for u in units} == {0, 1, 2, 3} and len(units) == 2304

    def check(i):
        u = units[i]
        box = oracle.narrow(_box(r, i))
        want, wk = oracle.compress_payload(box, r["keep"])
        if _payload(p, i) != want or int(p["kept"][i]) != wk:
            return i, "payload"
        back = oracle.decompress_payload(want)
        o = r["offs"][i]
        if p["regen"][o:o + u.cells].tobytes() != back.ravel().tobytes():
            return i, "regen"
        ref = oracle.rmse(box, back)
        if abs(float(p["rmse"][i]) - ref) > 1e-12 * abs(ref):
            return i, ("rmse", float(p["rmse"][i]), ref)
        return None

    with ThreadPoolExecutor(_threads()) as ex:
        bad = [x for x in ex.map(check, range(len(units))) if x is not None]
    assert not bad, bad[:16]
    frac = p["kept"].astype(np.int64).sum() / sum(u.cells for u in units)
    assert 0.05 < frac < 0.95


def test_c3_row_index_of_every_unit(c3_run):
    """The forward's row index, entry for entry, as the restatement derives it
    from each payload (tests/numpy_ref.py row_index); every C3 shape is
    row-indexable (even W, H and D % 8 == 0)."""
    import numpy_ref as R
    r = c3_run
    p = r["rows"]
    ent = 0
    for i, u in enumerate(r["units"]):
        assert u.W % 2 == 0 and u.H % 2 == 0 and u.D % 8 == 0
        want = R.row_index(_payload(p, i), u.W, u.H, u.D)
        assert np.array_equal(p["rowinfo"][ent:ent + u.W * u.H + 1], want), (i, u)
        ent += u.W * u.H + 1
    assert ent * 8 == p["rowinfo"].nbytes


def test_c3_paths_identical(c3_run):
    """The three round-trip forms give the same payloads, offsets, kept counts
    and cells; the two fused forms the same RMSE bits, the separate calls an
    RMSE within 1e-12 (another summation order)."""
    r = c3_run
    a, b, c = r["rows"], r["fused"], r["separate"]
    for x in (b, c):
        assert np.array_equal(a["offsets"], x["offsets"]) and np.array_equal(a["kept"], x["kept"])
        assert a["regen"].tobytes() == x["regen"].tobytes()
    for i in range(len(r["units"])):
        assert _payload(a, i) == _payload(b, i) == _payload(c, i), i
    assert np.array_equal(a["rmse"], b["rmse"])
    assert np.allclose(a["rmse"], c["rmse"], rtol=1e-12, atol=0)
    hdr_ok = all(np.frombuffer(_payload(a, i)[:20], "<i4").tolist() == [u.W, u.H, u.D, u.cells, int(a["kept"][i])]
                 for i, u in enumerate(r["units"]))
    assert hdr_ok
