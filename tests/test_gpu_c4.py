"""BASELINE.json configs[3] (C4) on one GPU, checked against the CPU oracle.

C4 = 10 timesteps x the C3 4-level AMR layout x 8 components = 46,080 units
(bench_workloads.WORKLOADS["c4"], fp64, keep 0.999f) in ONE wc_forward:
  * every unit: header (W, H, D, ncoeff, nrle) and 0 <= kept <= ncoeff;
  * payload bytes equal the oracle's (the reference's compress(),
    src/compressor.cpp:192-248, without xz) on >= 2 units of every (level,
    component, shape), plus units of the mean-0 components 3 and 7 whose signed
    max is negative (thresh < 0: every coefficient kept, src/compressor.cpp:
    212-226) — the re-staging fallback (k_transform_fallback) at scale;
  * the opt-in global-threshold mode (shard.global_threshold on one rank: stage,
    4096-bin histogram, threshold, one emit) keeps exactly the histogram's
    retained count, and sampled payloads equal the reference's mask + RLE +
    serialize at that threshold (oracle.compress_payload_thresh).
The reference's own loop runs these units one by one (src/modes.cpp:100-103).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KEEP = float(np.float32(0.999))


@pytest.fixture(scope="module")
def c4_run(wc):
    import torch
    import bench_workloads as bw
    units = bw.WORKLOADS["c4"]["units"]()
    assert len(units) == 46080
    dev = torch.device("cuda", 0)
    cells, offs, extent = bw.synth_cells(torch, dev, units, "f64")
    tab, n, _ = bw.units_array(wc.capi, units, offs)
    ctx = wc.capi.Context(0)
    cap = wc.capi.payload_bound(tab, n)
    payload = torch.empty(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    ctx.forward(cells.data_ptr(), wc.capi.WC_F64, tab, n, KEEP, payload.data_ptr(), cap, offsets.data_ptr(),
                kept.data_ptr())
    ctx.synchronize()
    r = dict(units=units, offs=offs, cells=cells, payload=payload, offsets_dev=offsets,
             offsets=offsets.cpu().numpy(), kept=kept.cpu().numpy(), tab=tab, n=n, ctx=ctx, dev=dev, cap=cap,
             kept_dev=kept)
    yield r
    ctx.close()
    del r, cells, payload
    torch.cuda.empty_cache()


def _box(r, oracle, i):
    u = r["units"][i]
    o = r["offs"][i]
    return oracle.narrow(r["cells"][o:o + u.cells].cpu().numpy().reshape(u.D, u.H, u.W))


def _payload(r, i, offsets=None, kept=None):
    offsets = r["offsets"] if offsets is None else offsets
    kept = r["kept"] if kept is None else kept
    po = int(offsets[i])
    return r["payload"][po:po + 20 + 8 * int(kept[i])].cpu().numpy().tobytes()


def _sample(units, per_group=2, seed=7):
    rng = np.random.default_rng(seed)
    groups = {}
    for i, u in enumerate(units):
        groups.setdefault((u.lev, u.comp, (u.W, u.H, u.D)), []).append(i)
    out = []
    for key in sorted(groups):
        idx = groups[key]
        out += [idx[0], idx[-1]] + list(rng.choice(idx[1:-1], size=min(per_group - 2, len(idx) - 2), replace=False))
    return sorted(set(out)), len(groups)


def test_c4_every_unit_header_and_kept(c4_run):
    import torch
    r = c4_run
    units = r["units"]
    n = r["n"]
    # the 20 header bytes of every unit, gathered on the device
    idx = r["offsets_dev"][:n].view(n, 1) + torch.arange(20, device=r["dev"]).view(1, 20)
    hdr = r["payload"][idx.reshape(-1)].cpu().numpy().reshape(n, 20).copy().view("<i4")
    want = np.array([[u.W, u.H, u.D, u.cells] for u in units], np.int32)
    assert np.array_equal(hdr[:, :4], want)
    assert np.array_equal(hdr[:, 4], r["kept"].astype(np.int32))
    cells = want[:, 3].astype(np.int64)
    assert np.all(r["kept"] >= 0) and np.all(r["kept"].astype(np.int64) <= cells)
    # the slots are the worst-case prefix (include/wavelet_amd.h): offsets[u] = 4 + sum(24 + 8 cells)
    slots = 4 + np.concatenate([[0], np.cumsum(24 + 8 * cells)[:-1]])
    assert np.array_equal(r["offsets"][:n].astype(np.int64), slots)
    frac = r["kept"].sum() / cells.sum()
    assert 0.05 < frac < 0.95


def test_c4_payloads_match_oracle(c4_run, oracle):
    r = c4_run
    units = r["units"]
    sample, ngroups = _sample(units)
    assert ngroups == 5 * 8  # (level, shape): L0, L1, L2 one shape each, L3 two; 8 components
    # units of the mean-0 components whose signed max is negative: every coefficient kept
    allkept = [i for i, u in enumerate(units) if u.comp in (3, 7) and int(r["kept"][i]) == u.cells]
    assert len(allkept) > 0, "no negative-max unit in C4 components 3/7"
    sample = sorted(set(sample) | set(allkept[:: max(1, len(allkept) // 12)][:12]))
    negative_max_seen = 0
    for i in sample:
        box = _box(r, oracle, i)
        want, wk = oracle.compress_payload(box, KEEP)
        assert _payload(r, i) == want, (i, units[i])
        assert int(r["kept"][i]) == wk
        flat = oracle.wavelet_decompose(box).ravel()
        mag = np.abs(flat.astype(np.float64))
        if flat[int(np.argmax(mag))] < 0:
            negative_max_seen += 1
            assert wk == units[i].cells  # thresh < 0: everything kept
    assert negative_max_seen > 0


def test_c4_global_threshold_mode(c4_run, oracle):
    import torch
    from wavelet_compression_amd.shard import global_threshold
    r = c4_run
    ctx, n, tab = r["ctx"], r["n"], r["tab"]
    hist = torch.zeros(4096, dtype=torch.int64, device=r["dev"])
    t, retained = global_threshold(ctx, r["cells"].data_ptr(), 1, tab, n, 0.7, hist)
    ctx.forward_emit(tab, n, 0.0, t, r["payload"].data_ptr(), r["cap"], r["offsets_dev"].data_ptr(),
                     r["kept_dev"].data_ptr())
    ctx.synchronize()
    kept = r["kept_dev"].cpu().numpy()
    offs = r["offsets_dev"].cpu().numpy()
    total = sum(u.cells for u in r["units"])
    assert int(kept.astype(np.int64).sum()) == retained
    assert retained >= total - int(np.floor(0.7 * total))
    sample, _ = _sample(r["units"], per_group=2, seed=11)
    for i in sample[::3]:
        assert _payload(r, i, offs, kept) == oracle.compress_payload_thresh(_box(r, oracle, i), t), i
