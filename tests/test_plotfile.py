"""Plotfile reading against the reference's own fixtures.

The reference's tests/plt0007{4,5} are read IN PLACE from /root/reference when
that directory exists (this container); they are not copied into the repo
(see DESIGN.md "Oracle and fixtures").  Expectations restate the reference's
Preprocessing test (src/preprocess.cpp:311-377) and String cleaning test
(src/argparse.cpp:181-187)."""
import os
from pathlib import Path

import numpy as np
import pytest

REF_TESTS = Path("/root/reference/tests")
needs_ref = pytest.mark.skipif(not (REF_TESTS / "plt00074" / "Header").exists(),
                               reason="reference fixtures not present on this host")


def test_clean_string(wc):
    from wavelet_compression_amd import plotfile as pf
    assert pf.clean_string("plt07400") == 7400
    assert pf.clean_string("fff9909") == 9909
    assert pf.clean_string("doctest.h") == -1
    assert pf.format_levels(1, 3) == [1, 2, 3]


@needs_ref
def test_preprocessing_expectations(wc):
    from wavelet_compression_amd import plotfile as pf
    files = [str(REF_TESTS / "plt00074"), str(REF_TESTS / "plt00075")]
    d = pf.preprocess_data(files, ["temp", "pressure"], [0, 1])
    b1 = d.boxes[0][1][0][0].astype(np.float32)   # time 0, level 1, box 0, comp 0
    b2 = d.boxes[1][0][1][1].astype(np.float32)   # time 1, level 0, box 1, comp 1
    assert b1.shape == (64, 32, 16) and np.all(b1 == np.float32(3902.4))
    assert b2.shape == (2, 4, 8) and np.all(b2 == np.float32(16.0))
    assert d.locations[0][0][0] == [0, 0, 0] and d.locations[1][1][1] == [16, 32, 64]
    assert d.dimensions[0][1][0] == [16, 32, 64] and d.dimensions[1][0][1] == [8, 4, 2]
    assert d.box_counts == [[2, 2], [2, 2]]
    assert d.min_values == [np.float32(16.0)] * 2 and d.max_values == [np.float32(3902.4)] * 2
    h0, h1 = d.headers
    assert h0.prob_lo + h0.prob_hi == [0.6, 0.5, 0.4, 0.8, 0.9, 1.0]
    assert h0.ref_ratios == [2]  # reference reads `dim` entries from this line; one is present
    assert abs(h0.time - 0.2219392) < 1e-9 and abs(h1.time - 0.3874982) < 1e-9
    assert [h0.level_steps, h1.level_steps] == [[1200, 1500], [1800, 2000]]
    assert h0.domain_dims == (256, 512, 256)


@needs_ref
def test_format_files(wc, tmp_path):
    from wavelet_compression_amd import plotfile as pf
    files = pf.format_files(str(REF_TESTS), "plt00074", "plt00075")
    assert [os.path.basename(f) for f in files] == ["plt00074", "plt00075"]
    assert [os.path.basename(f) for f in pf.format_files(str(REF_TESTS), "plt00075", "plt00075")] == ["plt00075"]
