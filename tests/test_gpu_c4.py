"""BASELINE.json configs[3] (C4) on one GPU, checked against the CPU oracle.

C4 = 10 timesteps x the C3 4-level AMR layout x 8 components = 46,080 units
(bench_workloads.WORKLOADS["c4"], fp64, keep 0.999f) in ONE wc_forward:
  * every unit: header (W, H, D, ncoeff, nrle) and 0 <= kept <= ncoeff;
  * EVERY unit's payload bytes and kept count equal the oracle's (the
    reference's compress(), src/compressor.cpp:192-248, without xz), streamed
    to the host in chunks and checked on a 16-thread pool; among them the
    units of the mean-0 components 3 and 7 whose signed max is negative
    (thresh < 0: every coefficient kept, src/compressor.cpp:212-226) — the
    re-staging fallback (k_transform_fallback) at scale;
  * the opt-in global-threshold mode (shard.global_threshold on one rank: stage,
    4096-bin histogram, threshold, one emit) keeps exactly the histogram's
    retained count, and EVERY unit's payload equals the reference's mask + RLE +
    serialize at that threshold (oracle.compress_payload_thresh).
The reference's own loop runs these units one by one (src/modes.cpp:100-103).
"""
import os
from concurrent.futures import ThreadPoolExecutor

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


def _threads():
    return max(1, min(16, os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))


def _chunks(units, max_cells=1 << 26):
    """Contiguous unit ranges of at most max_cells cells (one unit at least)."""
    a, n = 0, len(units)
    while a < n:
        b, c = a, 0
        while b < n and (b == a or c + units[b].cells <= max_cells):
            c += units[b].cells
            b += 1
        yield a, b
        a = b


def _check_every_unit(r, oracle, offsets, kept, want):
    """Every unit's payload bytes (and kept count) against want(narrowed box) ->
    (bytes, kept or None).  The cells and the payload span of a chunk of units
    cross to the host while the pool checks the chunks before it."""
    units, offs = r["units"], r["offs"]
    bad, pending = [], []
    with ThreadPoolExecutor(_threads()) as ex:
        for a, b in _chunks(units):
            c0 = offs[a]
            cells = r["cells"][c0:offs[b - 1] + units[b - 1].cells].cpu().numpy()
            p0 = int(offsets[a])
            pay = r["payload"][p0:int(offsets[b - 1]) + 20 + 8 * int(kept[b - 1])].cpu().numpy()

            def check(i, cells=cells, pay=pay, c0=c0, p0=p0):
                u = units[i]
                o = offs[i] - c0
                w, wk = want(oracle.narrow(cells[o:o + u.cells].reshape(u.D, u.H, u.W)))
                po = int(offsets[i]) - p0
                got = pay[po:po + 20 + 8 * int(kept[i])].tobytes()
                return None if (got == w and (wk is None or wk == int(kept[i]))) else i

            pending.append(ex.map(check, range(a, b)))  # submitted now, collected below
            while len(pending) > 2:  # bound the host copies in flight
                bad += [i for i in pending.pop(0) if i is not None]
        for p in pending:
            bad += [i for i in p if i is not None]
    return bad


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


def test_c4_every_payload_matches_oracle(c4_run, oracle):
    """All 46,080 forward payloads and kept counts against the oracle."""
    r = c4_run
    bad = _check_every_unit(r, oracle, r["offsets"], r["kept"], lambda box: oracle.compress_payload(box, KEEP))
    assert not bad, (len(bad), bad[:16])


def test_c4_negative_max_units_keep_everything(c4_run, oracle):
    """The sign quirk at scale: units of the mean-0 components whose first
    max-|c| coefficient is negative keep every coefficient (thresh < 0); their
    bytes are among those checked above, this pins that they exist in C4."""
    r = c4_run
    units = r["units"]
    _, ngroups = _sample(units)
    assert ngroups == 5 * 8  # (level, shape): L0, L1, L2 one shape each, L3 two; 8 components
    allkept = [i for i, u in enumerate(units) if u.comp in (3, 7) and int(r["kept"][i]) == u.cells]
    assert len(allkept) > 0, "no negative-max unit in C4 components 3/7"
    negative_max_seen = 0
    for i in allkept[:: max(1, len(allkept) // 12)][:12]:
        flat = oracle.wavelet_decompose(_box(r, oracle, i)).ravel()
        if flat[int(np.argmax(np.abs(flat.astype(np.float64))))] < 0:
            negative_max_seen += 1
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
    bad = _check_every_unit(r, oracle, offs, kept, lambda box: (oracle.compress_payload_thresh(box, t), None))
    assert not bad, (len(bad), bad[:16])
