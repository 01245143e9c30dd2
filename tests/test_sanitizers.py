"""Sanitizer builds of the host side (CPU, no GPU): the reference builds its
Debug configuration with -fsanitize=address (reference CMakeLists.txt:67-72);
here the host library, the CLI and the host-IO test are rebuilt with ASan +
UBSan (`make asan`) and with TSan (`make tsan`) and run over the host-only
paths: the xz thread pool (parallel encode == serial bytes, decode round trip,
presets 0/1/6 across 4 encode and 3 decode threads), plotfile read/write and
the reference fixtures, .raw side files, parameters, file selection, the
CLI's argument errors, and the core library's host pool + destination
prefault of the _host entry points (csrc/wc_hostmem.cpp, tests/cpp/
test_hostmem.cpp), and the _host entry points' pipeline itself (csrc/
wc_hostpipe.cpp + wc_common.cpp) over a CPU fake of the HIP runtime with
injected failures (tests/cpp/test_hostpipe.cpp).  Any sanitizer report fails
the test (halt_on_error)."""
import lzma
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "wavelet-compression_amd" / "csrc"
REF_TESTS = Path("/root/reference/tests")
SANS = ("asan", "tsan")


@pytest.fixture(scope="module")
def san_bins():
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(["make", "-s", "-j", jobs, "-C", str(CSRC), *SANS], check=True, timeout=900)
    return {s: ROOT / "tools" / "bin" / s for s in SANS}


def san_env(tmp_path):
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "halt_on_error=1:detect_leaks=1:abort_on_error=0:exitcode=66"
    env["UBSAN_OPTIONS"] = "halt_on_error=1:print_stacktrace=1:exitcode=66"
    env["TSAN_OPTIONS"] = "halt_on_error=1:exitcode=66"
    env["TMPDIR"] = str(tmp_path)
    return env


def check_clean(r, what):
    text = r.stdout + r.stderr
    assert "Sanitizer" not in text and "runtime error:" not in text, f"{what}:\n{text[-4000:]}"
    assert r.returncode != 66, f"{what}: sanitizer exit\n{text[-4000:]}"


@pytest.mark.parametrize("san", SANS)
def test_host_io_under_sanitizer(san_bins, san, tmp_path):
    args = [str(san_bins[san] / "test_host_io")]
    if (REF_TESTS / "plt00074" / "Header").exists():
        args.append(str(REF_TESTS))
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=san_env(tmp_path))
    check_clean(r, f"{san} test_host_io")
    assert r.returncode == 0 and "checks passed" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("san", SANS)
def test_xz_pool_presets_under_sanitizer(san_bins, san, tmp_path, oracle):
    """Oracle payloads through the pooled xz encoder/decoder at presets 0, 1, 6."""
    keep = 0.999
    want = {}
    for i, d in enumerate([(32, 32, 32), (16, 32, 64), (48, 32, 16), (8, 4, 2), (0, 4, 4)]):
        box = oracle.narrow(oracle.synth_box_f64(oracle.unit_seed(0, 0, i, 3), (0, 0, 0), *d))
        p, _ = oracle.compress_payload(box, keep)
        want[f"u{i}"] = p
        (tmp_path / f"u{i}.bin").write_bytes(p)
    r = subprocess.run([str(san_bins[san] / "test_host_io"), "--xz-presets", str(tmp_path), "0", "1", "6"],
                       capture_output=True, text=True, timeout=600, env=san_env(tmp_path))
    check_clean(r, f"{san} xz presets")
    assert r.returncode == 0, r.stdout + r.stderr
    for name, p in want.items():
        for pr in (0, 1, 6):
            assert lzma.decompress((tmp_path / f"{name}.p{pr}.xz").read_bytes(), format=lzma.FORMAT_XZ) == p


@pytest.mark.parametrize("san", SANS)
def test_cli_argument_errors_under_sanitizer(san_bins, san, tmp_path):
    cli = str(san_bins[san] / "wavelet-compression")
    env = san_env(tmp_path)
    r = subprocess.run([cli], capture_output=True, text=True, timeout=120, env=env)
    check_clean(r, f"{san} cli no mode")
    assert "Specify a mode" in r.stderr
    r = subprocess.run([cli, f"compresseddir={tmp_path}/", "-d"], capture_output=True, text=True, timeout=120, env=env)
    check_clean(r, f"{san} cli missing params")
    assert "Missing out directory!" in r.stderr


@pytest.mark.parametrize("san", SANS)
def test_host_pool_and_prefault_under_sanitizer(san_bins, san, tmp_path):
    """wc_hostmem: every pool task runs once (0..15 workers, 0..5000 tasks, 60
    jobs back to back); populate_for_write changes no byte (written data, never
    touched zeros, unaligned edges, both the MADV_POPULATE_WRITE and the
    per-page touch path) and leaves every whole page of the range resident."""
    r = subprocess.run([str(san_bins[san] / "test_hostmem")], capture_output=True, text=True, timeout=300,
                       env=san_env(tmp_path))
    check_clean(r, f"{san} test_hostmem")
    assert r.returncode == 0 and "checks passed" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("san", SANS)
def test_host_pipeline_under_sanitizer(san_bins, san, tmp_path):
    """wc_forward_host / wc_inverse_host over the fake runtime (streams are
    threads, events order them, pageable copies block): 1..16 unit runs, 0..8
    host threads, pinned and pageable sources (bounce slots), a kernel-raised
    error in a pipelined call, and an injected failure of every runtime
    call and device entry point the pipeline makes, each followed by a freed
    caller buffer (no copy may outlive the call) and a clean call."""
    r = subprocess.run([str(san_bins[san] / "test_hostpipe")], capture_output=True, text=True, timeout=600,
                       env=san_env(tmp_path))
    check_clean(r, f"{san} test_hostpipe")
    assert r.returncode == 0 and " 0 failed" in r.stdout, r.stdout + r.stderr
