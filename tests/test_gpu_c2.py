"""BASELINE.json configs[1] (C2, the headline workload) at full size on one GPU,
checked against the CPU oracle on EVERY unit: all 1024 x 64^3 fp64 boxes
(bench_workloads.WORKLOADS["c2"], the cells bench.py times) at keep 0.999f in
ONE wc_forward, then ONE wc_inverse_rmse of the payloads:
  * every unit's payload bytes equal the oracle's compress() minus xz
    (narrow + wavelet_decompose + signed max + mask + rle_encode + serialize,
    src/compressor.cpp:85-248), and its kept count;
  * every unit's reconstruction equals the oracle's decompress() minus xz
    (rle_decode + inverse_wavelet_decompose, src/decompressor.cpp:14-159) bit
    for bit, and its RMSE is within 1e-12 of calc_rmse_per_box on it
    (src/calc-loss.cpp:12-43 via the oracle).
The oracle runs on a thread pool (ctypes releases the GIL), so the whole batch
is checked in seconds.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEEP = float(np.float32(0.999))
N3 = 64 ** 3


@pytest.fixture(scope="module")
def c2_run(wc, ctx):
    import torch
    import bench_workloads as bw
    units = bw.WORKLOADS["c2"]["units"]()
    assert len(units) == 1024 and all(u.cells == N3 for u in units)
    dev = torch.device("cuda", 0)
    cells, offs, extent = bw.synth_cells(torch, dev, units, "f64")
    tab, n, _ = bw.units_array(wc.capi, units, offs)
    cap = wc.capi.payload_bound(tab, n)
    payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    regen = torch.full((extent,), float("nan"), dtype=torch.float32, device=dev)
    rmse = torch.full((n,), -1.0, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()  # the fills ran on torch's stream, the context has its own
    ctx.forward(cells.data_ptr(), wc.capi.WC_F64, tab, n, KEEP, payload.data_ptr(), cap, offsets.data_ptr(),
                kept.data_ptr())
    ctx.inverse_rmse(payload.data_ptr(), offsets.data_ptr(), tab, n, cells.data_ptr(), wc.capi.WC_F64,
                     regen.data_ptr(), rmse.data_ptr())
    ctx.synchronize()
    r = dict(n=n, offs=offs, offsets=offsets.cpu().numpy(), kept=kept.cpu().numpy(),
             cells=cells.cpu().numpy(), payload=payload.cpu().numpy(), regen=regen.cpu().numpy(),
             rmse=rmse.cpu().numpy())
    del cells, payload, offsets, kept, regen, rmse
    torch.cuda.empty_cache()
    return r


def _threads():
    return max(1, min(16, os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def _box(r, i):
    o = int(r["offs"][i])
    return r["cells"][o:o + N3].reshape(64, 64, 64)


def _payload(r, i):
    po = int(r["offsets"][i])
    return r["payload"][po:po + 20 + 8 * int(r["kept"][i])].tobytes()


def test_c2_every_payload_matches_oracle(c2_run, oracle):
    r = c2_run

    def check(i):
        want, k = oracle.compress_payload(oracle.narrow(_box(r, i)), KEEP)
        return i if (_payload(r, i) != want or int(r["kept"][i]) != k) else None

    with ThreadPoolExecutor(_threads()) as ex:
        bad = [i for i in ex.map(check, range(r["n"])) if i is not None]
    assert not bad, bad[:16]
    frac = r["kept"].astype(np.int64).sum() / (r["n"] * N3)
    assert 0.2 < frac < 0.4  # ~30 % kept at keep 0.999


def test_c2_every_reconstruction_and_rmse_match_oracle(c2_run, oracle):
    r = c2_run

    def check(i):
        want = oracle.decompress_payload(_payload(r, i))
        o = int(r["offs"][i])
        got = r["regen"][o:o + N3]
        if got.tobytes() != want.tobytes():
            return i, "regen"
        w = oracle.rmse(oracle.narrow(_box(r, i)), want)
        if abs(float(r["rmse"][i]) - w) > 1e-12 * abs(w):
            return i, ("rmse", float(r["rmse"][i]), w)
        return None

    with ThreadPoolExecutor(_threads()) as ex:
        bad = [x for x in ex.map(check, range(r["n"])) if x is not None]
    assert not bad, bad[:16]
