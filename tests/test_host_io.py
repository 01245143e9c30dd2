"""Host-side rows of the drop-in, no GPU needed:
.raw side files, plotfile reader and writer, the ParmParse-style parameters,
file selection and the xz thread pool, through tests/cpp/test_host_io.cpp
(the reference's own readandwrite / argparse / Preprocessing / Writing
plotfiles tests, restated).  The reference's fixtures tests/plt0007{4,5} are
read in place when /root/reference is present (this container) and those
cases skip elsewhere."""
import filecmp
import os
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "tools" / "bin" / "test_host_io"
CLI = ROOT / "wavelet-compression_amd" / "bin" / "wavelet-compression"
REF_TESTS = Path("/root/reference/tests")


def test_host_io_cpp_cases():
    args = [str(BIN)] + ([str(REF_TESTS)] if (REF_TESTS / "plt00074" / "Header").exists() else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checks passed" in r.stdout


@pytest.mark.skipif(not (REF_TESTS / "plt00074" / "Header").exists(), reason="reference fixtures not present")
def test_python_plotfile_writer_matches_reference_fixture(tmp_path):
    """The Python writer (used by the GPU tests to build inputs) reproduces the
    reference's tests/plt00074 byte for byte (src/writeplotfile.cpp:315-402 data)."""
    from wavelet_compression_amd import plotfile as pf
    b1 = np.full((2, 64, 32, 16), np.float32(3902.4), np.float64)
    b2 = np.full((2, 2, 4, 8), 16.0)
    lev = [((0, 0, 0), b1), ((16, 32, 64), b2)]
    for name, t, steps in (("plt00074", 0.2219392, [1200, 1500]), ("plt00075", 0.3874982, [1800, 2000])):
        pf.write_plotfile(tmp_path / name, ["temp", "pressure"], t, [0.6, 0.5, 0.4, 0.8, 0.9, 1.0], 2,
                          (256, 512, 256), steps, [lev, lev])
        ref = REF_TESTS / name
        for root, _, files in os.walk(ref):
            for f in files:
                a = Path(root) / f
                assert filecmp.cmp(a, tmp_path / name / a.relative_to(ref), shallow=False), a


def test_cli_without_mode_reports_error():
    r = subprocess.run([str(CLI)], capture_output=True, text=True, timeout=60)
    assert "Specify a mode" in r.stderr


def test_cli_reports_missing_parameters(tmp_path):
    """Missing parameters are logged, like ParmParse queries in src/argparse.cpp:17-68."""
    r = subprocess.run([str(CLI), f"compresseddir={tmp_path}/", "-d"], capture_output=True, text=True, timeout=60)
    assert "Missing out directory!" in r.stderr


def test_fast_xz_preset_decodes_to_oracle_payloads(tmp_path, oracle):
    """SURVEY §8(f) row 1's optional faster preset: oracle payloads of synthetic
    boxes, xz-encoded by the host pool at presets 0, 1 and 6, are read back by
    the reference-style stream decoder (host xz_decompress, src/decompressor.cpp:
    164-234) to the same payloads; preset 6 is byte-identical to liblzma's
    preset 6 / CRC64 (the reference's files); the fast presets are smaller than
    the payload and at most ~1.3x preset 6's size here."""
    import lzma
    keep = float(np.float32(0.999))
    want = {}
    for i, d in enumerate([(32, 32, 32), (16, 32, 64), (48, 32, 16), (8, 4, 2)]):
        box = oracle.narrow(oracle.synth_box_f64(oracle.unit_seed(0, 0, i, 0), (0, 0, 0), *d))
        p, _ = oracle.compress_payload(box, keep)
        want[f"u{i}"] = p
        (tmp_path / f"u{i}.bin").write_bytes(p)
    r = subprocess.run([str(BIN), "--xz-presets", str(tmp_path), "0", "1", "6"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    sizes = {}
    for line in r.stdout.split("\n"):
        if line.strip():
            name, pr, nb = line.split()
            sizes[(name, int(pr))] = int(nb)
    assert len(sizes) == 3 * len(want)
    for name, p in want.items():
        for pr in (0, 1, 6):
            blob = (tmp_path / f"{name}.p{pr}.xz").read_bytes()
            assert lzma.decompress(blob, format=lzma.FORMAT_XZ) == p, (name, pr)
        assert (tmp_path / f"{name}.p6.xz").read_bytes() == lzma.compress(
            p, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6), name
        if len(p) > 4096:
            assert sizes[(name, 0)] < len(p) and sizes[(name, 0)] <= 1.3 * sizes[(name, 6)], (name, sizes)
