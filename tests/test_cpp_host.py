"""The C++ mirror of the reference interface (include/wavelet_amd/*.h,
libwavelet_amd_host.so): exported signatures (CPU) and the reference's own
unit tests restated in tests/cpp/test_codec.cpp (GPU)."""
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
HOST_LIB = ROOT / "wavelet-compression_amd" / "lib" / "libwavelet_amd_host.so"
TEST_BIN = ROOT / "tools" / "bin" / "test_codec"

# The reference's public C++ API (src/compressor.h:9-15, src/decompressor.h:6-18,
# src/calc-loss.h:6-16), as demangled by nm -C.
REFERENCE_SIGNATURES = [
    "compress(std::vector<Grid3D<float>, std::allocator<Grid3D<float> > >&, std::vector<int, std::allocator<int> >, "
    "double, int, int, int, std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> >)",
    "decompress(std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> >, int, int, int, int)",
    "deserialize_compressed_wavelet(std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> > const&)",
    "inverse_wavelet_decompose(std::vector<float, std::allocator<float> >, int, int, int)",
    "calc_rmse_per_box(std::vector<Grid3D<float>, std::allocator<Grid3D<float> > > const&, "
    "std::vector<Grid3D<float>, std::allocator<Grid3D<float> > > const&, int)",
    "calc_adj_loss(double, double)",
    "calc_size(std::__cxx11::basic_string<char, std::char_traits<char>, std::allocator<char> >)",
]


def test_host_library_exports_reference_signatures():
    out = subprocess.run(["nm", "-DC", "--defined-only", str(HOST_LIB)], capture_output=True, text=True,
                         check=True).stdout
    for sig in REFERENCE_SIGNATURES:
        assert sig in out, sig


def test_host_library_links_codec_and_liblzma():
    out = subprocess.run(["ldd", str(HOST_LIB)], capture_output=True, text=True, check=True).stdout
    assert "libwavelet_amd.so" in out and "liblzma.so.5" in out


@pytest.mark.gpu
def test_reference_unit_tests_against_cpp_mirror():
    r = subprocess.run([str(TEST_BIN)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "7 cases" in r.stdout


@pytest.mark.gpu
def test_random_boxes_through_cpp_mirror():
    """tests/cpp/test_mirror_fuzz.cpp: seeded random multiBox3Ds (1-4 components,
    random dims up to 64 per axis, fields with NaN / inf / subnormals, random
    float32 keeps) through the C++ mirror's compress() / decompress() /
    calc_rmse_per_box against the CPU oracle compiled into that test binary:
    the returned pairs and the decoded boxes bit for bit, the files under the
    reference's names, the RMSE within the summation-order bound.
    WC_MIRROR_FUZZ_SEEDS overrides the 24 seeds (a longer soak)."""
    import os
    seeds = os.environ.get("WC_MIRROR_FUZZ_SEEDS", "24")
    r = subprocess.run([str(ROOT / "tools" / "bin" / "test_mirror_fuzz"), seeds], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert f"{seeds} seeds" in r.stdout
