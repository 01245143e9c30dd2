"""CPU pin of tests/tiled_expect.py: for boxes tiled from small seeded boxes,
the expected payload bytes and reconstruction built from the small box equal
the oracle's own compress()/decompress() of the tiled box (src/compressor.cpp:
85-248, src/decompressor.cpp:14-159).  The GPU maximum-size tests rest on it."""
import numpy as np
import pytest

from tiled_expect import TiledExpect, axis_map

KEEPS = [float(np.float32(k)) for k in (0.99, 0.999, 0.9999)]


def _small(O, dims, seed):
    W, H, D = dims
    return O.narrow(O.synth_box_f64(O.unit_seed(seed, 1, 2, 3), (5, 7, 11), W, H, D))


def test_axis_map_is_blockwise():
    m = axis_map(12, 4)
    # low half: blocks 0..5 -> 0,1,0,1,0,1; high half the same, shifted by n/2
    assert m.tolist() == [0, 1, 0, 1, 0, 1, 2, 3, 2, 3, 2, 3]


@pytest.mark.parametrize("small,reps", [((6, 4, 8), (2, 3, 1)), ((8, 6, 4), (3, 1, 2)), ((10, 8, 6), (2, 2, 3))])
@pytest.mark.parametrize("keep", KEEPS)
def test_tiled_expectation_matches_oracle(oracle, small, reps, keep):
    import torch
    b = _small(oracle, small, seed=sum(small))
    ex = TiledExpect(oracle, b, keep)
    W, H, D = small[0] * reps[0], small[1] * reps[1], small[2] * reps[2]
    big = np.tile(b, (reps[2], reps[1], reps[0]))
    assert big.shape == (D, H, W)
    want, k = oracle.compress_payload(big, keep)
    dev = torch.device("cpu")
    pairs = torch.cat(list(ex.pair_slabs(torch, dev, W, H, D, slab=4)))
    hdr = np.array([W, H, D, W * H * D, pairs.shape[0]], "<i4").tobytes()
    assert hdr + pairs.numpy().tobytes() == want
    assert pairs.shape[0] == k
    regen = torch.cat(list(ex.regen_slabs(torch, dev, W, H, D))).numpy()
    assert regen.tobytes() == oracle.decompress_payload(want).tobytes()
    assert oracle.rmse(big, regen) == pytest.approx(ex.rmse, rel=1e-12)
    tiled = ex.tiled(torch, b, dev, W, H, D).numpy()
    assert tiled.tobytes() == big.tobytes()
