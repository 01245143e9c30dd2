"""Pin the CPU oracle (oracle/wc_oracle.c) before trusting it as the checker.

Three independent anchors:
  1. the reference's own doctest known answers (src/compressor.cpp:300-406,
     src/calc-loss.cpp:68-86), restated here;
  2. goldens recorded in SURVEY.md §8(c) from the compiled reference (probe);
  3. a second restatement in numpy (tests/numpy_ref.py) on random boxes of
     many shapes, including odd dims, extreme magnitudes and NaN/inf.
Plus the committed golden fixtures (tests/golden/*.npz) must still reproduce.
"""
import hashlib
import lzma
import json
from pathlib import Path

import numpy as np
import pytest

import numpy_ref as NR

GOLDEN = Path(__file__).parent / "golden"
F999 = float(np.float32(0.999))


# ---- 1. the reference's own unit tests ------------------------------------

def test_rle_encode_truth_tables(oracle):
    """src/compressor.cpp:300-339."""
    values = [1.0, 2.0, 3.0, 4.0, 5.0]
    assert oracle.rle_encode([1, 1, 0, 0, 1], values) == [(0, 1.0), (0, 2.0), (2, 3.0)]
    assert oracle.rle_encode([1] * 5, values) == [(0, v) for v in values]
    assert oracle.rle_encode([0] * 5, values) == []


def test_serialization_round_trip(oracle, wc):
    """src/compressor.cpp:342-366 (with need32 compared as written, never serialized)."""
    rng = np.random.default_rng(5)
    W, H, D, nc = (int(v) for v in rng.integers(1, 101, 4))
    runs, vals = np.array([0, 0, 2], np.int32), np.array([1.0, 2.0, 3.0], np.float32)
    blob = oracle.serialize(W, H, D, nc, runs, vals)
    cw = wc.deserialize_compressed_wavelet(blob)
    assert cw.shape == [W, H, D] and cw.coeff_shape == [nc]
    assert cw.rle_encoded == [(0, 1.0), (0, 2.0), (2, 3.0)]
    assert cw.need32 is False
    assert wc.serialize_compressed_wavelet(cw) == blob


def test_wavelet_round_trip_4x8x16(oracle):
    """src/compressor.cpp:369-384: 4x8x16 box round trip within 1e-6."""
    box = np.full((16, 8, 4), 5.0, np.float32)
    for (x, y, z, v) in [(1, 2, 3, 8.5), (2, 5, 6, 5.44), (1, 1, 1, 3.3999932),
                         (2, 2, 2, 3.19229), (3, 5, 12, 199.39029)]:
        box[z, y, x] = np.float32(v)
    back = oracle.inverse_wavelet_decompose(oracle.wavelet_decompose(box), 4, 8, 16)
    assert np.all(np.abs(back - box) <= 1e-6)


def test_file_writing_const_box_exact(oracle, tmp_path):
    """src/compressor.cpp:387-406: const 5.0 box, keep 0.999, exact through xz."""
    box = np.full((16, 8, 4), 5.0, np.float32)
    payload, _ = oracle.compress_payload(box, 0.999)
    f = tmp_path / "compressed-wavelet-0-0-0-0.xz"
    f.write_bytes(lzma.compress(payload, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6))
    back = oracle.decompress_payload(lzma.decompress(f.read_bytes()))
    assert np.array_equal(back, box)


def test_calc_rmse(oracle):
    """src/calc-loss.cpp:68-86: {3.5, 3.5}."""
    a = np.zeros((2, 2, 2), np.float32)
    p = np.full((2, 2, 2), 3.5, np.float32)
    assert [oracle.rmse(a, p), oracle.rmse(a, p)] == [3.5, 3.5]


# ---- 2. SURVEY.md §8(c) goldens from the compiled reference ------------------

def test_survey_golden_8x4x2_const16(oracle):
    box = np.full((2, 4, 8), 16.0, np.float32)
    payload, kept = oracle.compress_payload(box, F999)
    assert len(payload) == 84 and kept == 8
    hdr = np.frombuffer(payload[:20], "<i4").tolist()
    assert hdr == [8, 4, 2, 64, 8]
    pairs = np.frombuffer(payload[20:], dtype=[("r", "<i4"), ("v", "<f4")])
    assert pairs["r"].tolist() == [0, 1, 5, 1, 5, 1, 5, 1]
    assert np.all(pairs["v"] == 16.0)
    assert len(lzma.compress(payload, format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64, preset=6)) == 88


def test_survey_golden_sign_quirk(oracle):
    spike = np.full((4, 4, 4), 5.0, np.float32)
    spike[1, 2, 3] = 7.5
    assert oracle.compress_payload(spike, F999)[1] == 15
    assert oracle.compress_payload(np.full((4, 4, 4), -5.0, np.float32), F999)[1] == 64


def test_survey_golden_keep_widening():
    assert 1 - float(np.float32(0.999)) == 0.00099998712539672852


def test_survey_golden_odd_tail_zero(oracle):
    box = np.full((2, 4, 3), 7.0, np.float32)  # 3x4x2
    back = oracle.decompress_payload(oracle.compress_payload(box, F999)[0])
    assert np.all(back[:, :, 2] == 0.0) and np.all(back[:, :, :2] == 7.0)


def test_survey_golden_const_3902(oracle):
    box = np.full((64, 32, 16), np.float32(3902.39990234375), np.float32)
    payload, kept = oracle.compress_payload(box, F999)
    assert kept == 4096
    assert np.array_equal(oracle.decompress_payload(payload), box)


# ---- 3. independent numpy restatement ---------------------------------------

SHAPES = [(2, 2, 2), (8, 4, 2), (6, 10, 14), (3, 4, 2), (3, 5, 7), (1, 1, 1), (1, 7, 1),
          (16, 16, 16), (16, 32, 64), (33, 17, 9), (66, 2, 13)]


@pytest.mark.parametrize("dims", SHAPES)
def test_oracle_matches_numpy_restatement(oracle, dims):
    W, H, D = dims
    rng = np.random.default_rng(W * 10007 + H * 101 + D)
    box = (rng.standard_normal((D, H, W)) * np.exp2(rng.integers(-20, 20, (D, H, W)))).astype(np.float32)
    flat = oracle.wavelet_decompose(box)
    assert flat.tobytes() == NR.wavelet_decompose(box).tobytes()
    for keep in (0.99, 0.999, 0.9999):
        k = float(np.float32(keep))
        assert oracle.compress_payload(box, k)[0] == NR.compress_payload(box, k)
    assert oracle.inverse_wavelet_decompose(flat, W, H, D).tobytes() == \
        NR.inverse_wavelet_decompose(flat, W, H, D).tobytes()


def test_oracle_matches_numpy_specials(oracle):
    rng = np.random.default_rng(3)
    for trial in range(6):
        box = rng.standard_normal((6, 4, 8)).astype(np.float32)
        if trial == 0:
            box[0, 0, 0] = np.nan          # NaN first -> thresh NaN -> nothing kept
        elif trial == 1:
            box[3, 2, 5] = np.nan
        elif trial == 2:
            box[1, 1, 1] = -np.inf
        elif trial == 3:
            box[:] = -2.0                  # negative max -> everything kept
        elif trial == 4:
            box *= np.float32(1e-41)       # subnormals
        else:
            box[2, 2, 2] = 3e38; box[2, 2, 3] = 3e38  # overflowing float adds
        for keep in (0.99, 0.999):
            k = float(np.float32(keep))
            assert oracle.compress_payload(box, k)[0] == NR.compress_payload(box, k), trial


def test_synth_generator_properties(oracle):
    """The SURVEY §8(d) field: smooth + sigma noise; kept fraction ~30 % at 64^3/0.999f."""
    b = oracle.synth_box_f64(oracle.unit_seed(0, 0, 0, 0), (0, 0, 0), 64, 64, 64)
    assert b.shape == (64, 64, 64) and 240 < b.mean() < 360
    _, kept = oracle.compress_payload(oracle.narrow(b), F999)
    assert 0.25 < kept / 64 ** 3 < 0.36


# ---- committed golden fixtures ----------------------------------------------

def test_golden_fixtures_reproduce(oracle):
    """tests/golden/codec_golden.npz (made by tests/golden/make_golden.py)."""
    z = np.load(GOLDEN / "codec_golden.npz")
    meta = json.loads((GOLDEN / "codec_golden.json").read_text())
    for case in meta["cases"]:
        name = case["name"]
        box = z[case["box"]]
        payload = z[name + "/payload"].tobytes()
        got, kept = oracle.compress_payload(box, case["keep"])
        assert got == payload, name
        assert kept == case["kept"], name
        assert oracle.decompress_payload(payload).tobytes() == z[name + "/regen"].tobytes(), name
    for h in meta["hashes"]:
        cells = oracle.synth_box_f64(h["seed"], h["lo"], *h["dims"])
        payload, _ = oracle.compress_payload(oracle.narrow(cells), h["keep"])
        assert hashlib.sha256(payload).hexdigest() == h["payload_sha256"], h["dims"]
