"""Property checks of the oracle (oracle/wc_oracle.c) against the independent
numpy restatement (tests/numpy_ref.py), over hypothesis-drawn boxes: random
dims (odd and even, 1..24 per axis), cell values from every float32 regime
(subnormal to near-overflow, both signs, exact ties, constants, with NaN / inf
sprinkled in) and random float32 keeps (the reference's Config::keep,
src/argparse.h:13), keeps >= 1 included (thresh <= 0: the sign quirk's
territory, src/compressor.cpp:212-226).  Every case: the flat coefficients
(src/compressor.cpp:85-185), the serialized payload (:192-248) and the
inverse of the flat array (src/decompressor.cpp:79-159) are identical byte
for byte, and decompress() of the payload equals the restatement's
rle_decode + inverse (src/decompressor.cpp:14-30).  CPU only.
"""
import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import numpy_ref as NR

DIM = st.integers(min_value=1, max_value=24)


@st.composite
def boxes(draw):
    W, H, D = draw(DIM), draw(DIM), draw(DIM)
    seed = draw(st.integers(min_value=0, max_value=2 ** 32 - 1))
    kind = draw(st.sampled_from(["normal", "wide", "tiny", "const", "ties", "specials"]))
    rng = np.random.default_rng(seed)
    if kind == "normal":
        b = rng.standard_normal((D, H, W)) * 10.0
    elif kind == "wide":
        b = rng.standard_normal((D, H, W)) * np.exp2(rng.integers(-120, 120, (D, H, W)))
    elif kind == "tiny":
        b = rng.standard_normal((D, H, W)) * 1e-42
    elif kind == "const":
        b = np.full((D, H, W), float(rng.choice([-1.0, 1.0]) * rng.uniform(0, 1e6)))
    elif kind == "ties":  # few distinct magnitudes: max_element's first-index rule decides
        b = rng.choice([-3.0, -1.0, 0.0, 1.0, 3.0], size=(D, H, W))
    else:
        b = rng.standard_normal((D, H, W))
        flat = b.reshape(-1)
        for v in (np.nan, np.inf, -np.inf, 3.0e38, -3.0e38):
            if rng.random() < 0.4:
                flat[rng.integers(0, flat.size)] = v
    keep = float(np.float32(draw(st.sampled_from([0.0, 0.5, 0.99, 0.999, 0.9999, 1.0, 1.5])
                                 | st.floats(min_value=0.0, max_value=1.0, width=32))))
    return b.astype(np.float32), keep


@settings(max_examples=300, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(boxes())
def test_oracle_equals_numpy_restatement(oracle, case):
    box, keep = case
    D, H, W = box.shape
    with np.errstate(all="ignore"):
        flat = oracle.wavelet_decompose(box)
        assert flat.tobytes() == NR.wavelet_decompose(box).tobytes()
        payload, kept = oracle.compress_payload(box, keep)
        assert payload == NR.compress_payload(box, keep)
        assert len(payload) == 20 + 8 * kept
        assert oracle.inverse_wavelet_decompose(flat, W, H, D).tobytes() == \
            NR.inverse_wavelet_decompose(flat, W, H, D).tobytes()
        (_, _, _), nc, runs, vals = oracle.parse_payload(payload)
        dense = np.zeros(W * H * D, np.float32)
        pos = np.cumsum(runs.astype(np.int64) + 1) - 1
        dense[pos[pos < nc]] = vals[pos < nc]
        assert oracle.decompress_payload(payload).tobytes() == \
            NR.inverse_wavelet_decompose(dense, W, H, D).tobytes()

