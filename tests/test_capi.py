"""The C-ABI library loads on a CPU-only host and exports every entry point
include/wavelet_amd.h declares; host-only helpers and argument checks work
without a GPU.  No compute call is made here (those are the -m gpu tests)."""
import ctypes
import re
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent


def declared_functions():
    text = (ROOT / "include" / "wavelet_amd.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(wc_[a-z_0-9]+)\s*\(", text)))


def test_header_declares_expected_entry_points(wc):
    decl = declared_functions()
    assert "wc_forward" in decl and "wc_inverse" in decl and "wc_rmse" in decl
    assert set(decl) == set(wc.capi.EXPORTED)


def test_binding_constants_match_header(wc):
    """Every status, dtype and option constant of include/wavelet_amd.h has the
    same value in the Python binding, the stage names follow the WC_STAGE_*
    indices, and HIST_BINS is WC_HIST_BINS: the binding cannot drift from the ABI."""
    import re
    from pathlib import Path
    text = (Path(__file__).resolve().parent.parent / "include" / "wavelet_amd.h").read_text()
    defs = {m.group(1): int(m.group(2)) for m in re.finditer(r"^#define (WC_[A-Z0-9_]+) (\d+)", text, re.M)}
    checked = 0
    for name, v in defs.items():
        if name.startswith(("WC_OK", "WC_ERR_", "WC_F32", "WC_F64", "WC_OPT_")):
            assert getattr(wc.capi, name) == v, name
            checked += 1
    assert checked >= 20
    stages = sorted((v, k) for k, v in defs.items() if k.startswith("WC_STAGE_"))
    assert len(stages) == defs["WC_NUM_STAGES"] == len(wc.capi.STAGES)
    for (i, k), s in zip(stages, wc.capi.STAGES):
        assert k == "WC_STAGE_" + s.upper(), (k, s)
    assert wc.capi.HIST_BINS == defs["WC_HIST_BINS"]


def test_library_exports_every_declared_symbol(wc):
    lib = wc.capi.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name


def test_shared_object_dynamic_symbols(wc):
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", str(wc.capi.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (wc_\w+)", out))
    assert set(declared_functions()) <= exported
    # only the boundary is exported with C linkage: no stray unmangled wc_ symbols
    assert exported == set(declared_functions())


def test_library_is_built_for_gfx950(wc):
    blob = wc.capi.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_host_helpers(wc):
    units, n, extent = wc.capi.make_units([(64, 64, 64), (8, 4, 2), (3, 5, 7)])
    L = wc.capi.load_library()
    assert L.wc_cell_count(units, n) == 64 ** 3 + 64 + 105
    assert L.wc_payload_bound(units, n) == 4 + sum(24 + 8 * c for c in (64 ** 3, 64, 105))
    assert units[1].cell_offset % 4 == 0 and units[2].cell_offset % 4 == 0
    assert L.wc_version().startswith(b"wavelet_amd")
    # row index: W*H + 1 entries of 8 B per unit with cells, none for an empty unit
    assert wc.capi.rowindex_bytes(units, n) == 8 * (64 * 64 + 1 + 8 * 4 + 1 + 3 * 5 + 1)
    e_units, e_n, _ = wc.capi.make_units([(0, 4, 4), (2, 2, 8), (1024, 1024, 0)])
    assert wc.capi.rowindex_bytes(e_units, e_n) == 8 * (2 * 2 + 1)


def test_null_context_is_rejected(wc):
    L = wc.capi.load_library()
    units, n, _ = wc.capi.make_units([(4, 4, 4)])
    assert L.wc_forward(None, None, 0, units, n, 0.999, None, 0, None, None) == wc.capi.WC_ERR_INVALID
    assert L.wc_inverse(None, None, None, units, n, None) == wc.capi.WC_ERR_INVALID
    assert L.wc_set_option(None, 1, 0) == wc.capi.WC_ERR_INVALID
    assert L.wc_last_error(None) == b"null context"


def test_context_creation_without_gpu_fails_loudly(wc):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(wc.WaveletError):
        wc.capi.Context(0)


def test_package_has_no_cpu_fallback():
    """The product never imports the oracle (test infrastructure only)."""
    pkg = ROOT / "wavelet-compression_amd"
    for f in list(pkg.glob("*.py")) + list((pkg / "csrc").rglob("*")):
        if f.is_file() and f.suffix in (".py", ".cpp", ".hip", ".h"):
            text = f.read_text()
            assert "oracle" not in text.replace("oracle/", "").lower() or f.name == "__init__.py", f


def test_hist_threshold_matches_restatement(wc, oracle):
    """wc_hist_threshold (host only) against the numpy restatement, including
    the empty histogram, quantile 0 / 1, bin 0 and the +inf bin."""
    rng = np.random.default_rng(7)
    cases = [np.zeros(4096, np.uint64)]
    h = np.zeros(4096, np.uint64)
    h[0] = 5
    h[4080] = 2  # +inf
    cases.append(h)
    for _ in range(6):
        h = np.zeros(4096, np.uint64)
        idx = rng.integers(0, 4096, 40)
        h[idx] = rng.integers(1, 10 ** 6, 40).astype(np.uint64)
        cases.append(h)
    for h in cases:
        for q in (0.0, 0.3, 0.5, 0.9, 0.999, 1.0):
            assert wc.capi.hist_threshold(h, q) == oracle.hist_threshold(h, q), (q, np.nonzero(h))
    with pytest.raises(wc.WaveletError):
        wc.capi.hist_threshold(np.zeros(4096, np.uint64), 1.5)


def test_hist_threshold_is_exact_on_coefficients(wc, oracle):
    """Keeping |c| > threshold retains exactly the histogram's retained count."""
    flat = oracle.wavelet_decompose(oracle.narrow(oracle.synth_box_f64(11, (0, 0, 0), 16, 8, 32)))
    h = oracle.magnitude_hist(flat)
    for q in (0.1, 0.7, 0.99):
        t, r = wc.capi.hist_threshold(h, q)
        assert int(np.count_nonzero(np.abs(flat) > np.float32(t))) == r


def test_no_kernel_spills_to_scratch(tmp_path):
    """Every shipped gfx950 kernel keeps its state in registers and LDS: code
    object metadata .private_segment_fixed_size == 0 and no VGPR spills
    (a private array indexed at run time or a spill would live in scratch; the
    round-2 four-tiles-per-block emit variant that faulted is the cautionary
    case, DESIGN.md §Forward progress)."""
    import re
    import subprocess
    from pathlib import Path
    llvm = Path("/opt/rocm/lib/llvm/bin")
    pkg = Path(__file__).resolve().parent.parent / "wavelet-compression_amd"
    kernels = {p.stem for p in (pkg / "csrc").glob("*.hip")}  # the .cpp objects are host code only
    objs = sorted(o for o in (pkg / "build").glob("wc_*.o") if o.stem in kernels)
    if not llvm.exists() or not objs:
        pytest.skip("ROCm LLVM tools or built objects absent")
    seen = 0
    for o in objs:
        fat, co = tmp_path / (o.stem + ".fat"), tmp_path / (o.stem + ".co")
        subprocess.run([str(llvm / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(o)], check=True)
        subprocess.run([str(llvm / "clang-offload-bundler"), "--type=o", "--unbundle", f"--input={fat}",
                        f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"], check=True)
        notes = subprocess.run([str(llvm / "llvm-readelf"), "--notes", str(co)], capture_output=True, text=True,
                               check=True).stdout
        for block in re.split(r"\n  - ", notes.split("amdhsa.kernels:", 1)[1])[1:]:
            m = re.search(r"\.name:\s+(\S+)", block)
            if not m:
                continue
            name = m.group(1)
            for key in ("private_segment_fixed_size", "vgpr_spill_count"):  # SGPR spills go to VGPR lanes
                m = re.search(r"\." + key + r":\s+(\d+)", block)
                assert m and int(m.group(1)) == 0, (o.name, name, key)
            seen += 1
    assert seen >= 20
