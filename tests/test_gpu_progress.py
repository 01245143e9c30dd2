"""Forward progress of the look-backs on a shared device (DESIGN.md §Forward
progress; VERDICT r2 "next" 6).

* A look-back wait that times out (forced here with WC_OPT_SPIN_LIMIT 1: the
  first unanswered poll fails) is reported as WC_ERR_HIP, makes the context's
  ticket form sticky, and later calls — also a second context's, in flight on
  its own stream at the same time — give the oracle's payloads without another
  ~2 s wait.
* The row-indexed inverse never reads past a payload when a timed-out row
  index would leave row entries of an earlier, denser batch behind (the
  timed-out row-index tile empties every row entry of its unit).
* WCAMD_SHARED_DEVICE=1 puts every context of a process on the tickets.
"""
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np
import pytest
from wavelet_compression_amd.capi import WC_OPT_ORDERED, WC_OPT_SPIN_LIMIT, WC_OPT_TICKETS

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
KEEP = float(np.float32(0.999))


def _boxes(oracle, n, dim, seed0):
    return [oracle.synth_box_f64(oracle.unit_seed(seed0, 0, i, 0), (dim * (i % 8), dim * (i // 8), 0), dim, dim, dim)
            for i in range(n)]


class DevBatch:
    """A batch of fp64 boxes resident on the device with its output buffers."""

    def __init__(self, wc, boxes):
        import torch
        dims = [(b.shape[2], b.shape[1], b.shape[0]) for b in boxes]
        self.units, self.n, self.extent = wc.capi.make_units(dims)
        host = np.zeros(self.extent, np.float64)
        for i, b in enumerate(boxes):
            o = self.units[i].cell_offset
            host[o:o + b.size] = b.ravel()
        dev = torch.device("cuda", 0)
        self.cells = torch.from_numpy(host).to(dev)
        self.cap = wc.capi.payload_bound(self.units, self.n)
        self.payload = torch.zeros(self.cap, dtype=torch.uint8, device=dev)
        self.offsets = torch.zeros(self.n + 1, dtype=torch.int64, device=dev)
        self.kept = torch.zeros(self.n, dtype=torch.int32, device=dev)
        self.out = torch.zeros(max(self.extent, 1), dtype=torch.float32, device=dev)
        torch.cuda.synchronize()

    def forward(self, wc, c):
        c.forward(self.cells.data_ptr(), wc.capi.WC_F64, self.units, self.n, KEEP, self.payload.data_ptr(),
                  self.cap, self.offsets.data_ptr(), self.kept.data_ptr())

    def inverse(self, c):
        c.inverse(self.payload.data_ptr(), self.offsets.data_ptr(), self.units, self.n, self.out.data_ptr())

    def payloads(self):
        p = self.payload.cpu().numpy()
        o = self.offsets.cpu().numpy()
        k = self.kept.cpu().numpy()
        return [p[int(o[i]):int(o[i]) + 20 + 8 * int(k[i])].tobytes() for i in range(self.n)]


def _force_timeout(wc, c, step, tries=6):
    """Run `step` under WC_OPT_SPIN_LIMIT 1 until a look-back wait times out
    (WC_ERR_HIP at the synchronisation); returns whether one did."""
    c.set_option(WC_OPT_SPIN_LIMIT, 1)
    try:
        for _ in range(tries):
            step()
            try:
                c.synchronize()
            except wc.WaveletError as e:
                assert e.code == wc.capi.WC_ERR_HIP and "timed out" in str(e), e
                return True
        return False
    finally:
        c.set_option(WC_OPT_SPIN_LIMIT, 0)


def test_timeout_makes_tickets_sticky_and_second_context_runs(wc, ctx, oracle):
    boxes = _boxes(oracle, 256, 64, seed0=41)
    want = [oracle.compress_payload(oracle.narrow(b), KEEP)[0] for b in boxes]
    b1 = DevBatch(wc, boxes)
    ctx.set_option(WC_OPT_TICKETS, 0)
    # launch order unless another live context of this process shares the device
    ordered0 = ctx.get_option(WC_OPT_ORDERED)
    try:
        assert _force_timeout(wc, ctx, lambda: b1.forward(wc, ctx)), "no look-back wait in 6 batches"
        assert ctx.get_option(WC_OPT_TICKETS) == 1 and ctx.get_option(WC_OPT_ORDERED) == 0  # sticky
        # the same context again, and a second context concurrently on its own stream
        other = wc.capi.Context(0)
        try:
            b2 = DevBatch(wc, boxes[:128])
            t0 = time.perf_counter()
            for _ in range(3):
                b1.forward(wc, ctx)
                b2.forward(wc, other)
            ctx.synchronize()
            other.synchronize()
            dt = time.perf_counter() - t0
            assert dt < 1.5, f"{dt:.2f} s: a look-back waited out its bound again"
            assert b1.payloads() == want
            assert b2.payloads() == want[:128]
        finally:
            other.close()
        assert ctx.get_option(WC_OPT_ORDERED) == 0  # still sticky after the other context left
    finally:
        ctx.set_option(WC_OPT_TICKETS, 0)
    assert ctx.get_option(WC_OPT_ORDERED) == ordered0


def test_host_entry_point_retries_after_timeout(wc, ctx, oracle):
    """wc_forward_host re-runs a call whose launch-order look-back timed out
    with the tickets (sticky afterwards) and returns the oracle's bytes."""
    from test_gpu_parity import pack
    boxes = _boxes(oracle, 64, 64, seed0=43)
    units, n, extent, cells = pack(wc, boxes)
    b1 = DevBatch(wc, boxes)
    ctx.set_option(WC_OPT_TICKETS, 0)
    try:
        assert _force_timeout(wc, ctx, lambda: b1.forward(wc, ctx))
        ctx.set_option(WC_OPT_TICKETS, 0)  # launch order again; the host call times out, retries with tickets
        ctx.set_option(WC_OPT_SPIN_LIMIT, 1)
        try:
            try:
                payload, offs, kept = ctx.forward_host(cells, units, n, KEEP)
                ok = True
            except wc.WaveletError as e:  # the retry (tickets) may time out too under a 1-poll bound
                assert e.code == wc.capi.WC_ERR_HIP
                ok = False
        finally:
            ctx.set_option(WC_OPT_SPIN_LIMIT, 0)
        if not ok:
            payload, offs, kept = ctx.forward_host(cells, units, n, KEEP)
        for i, b in enumerate(boxes):
            assert wc.capi.unit_payload(payload, offs, kept, i) == oracle.compress_payload(oracle.narrow(b), KEEP)[0]
    finally:
        ctx.set_option(WC_OPT_TICKETS, 0)


def test_inverse_timeout_never_reads_past_payload(wc, ctx, oracle):
    """Row entries of an earlier, denser batch are left in the context's row
    index; an inverse of sparser payloads whose row-index look-backs time out
    must not fault (the timed-out tile empties its unit's row entries), reports
    WC_ERR_HIP, and the next inverse (tickets) reconstructs exactly."""
    dense = _boxes(oracle, 64, 64, seed0=45)
    bd = DevBatch(wc, dense)
    bd.forward(wc, ctx)
    ctx.synchronize()
    bd.inverse(ctx)  # rowinfo now holds this batch's entries
    ctx.synchronize()
    # a batch with the same units whose payloads are nearly empty (constant boxes)
    flat = [np.full(b.shape, 7.0) for b in dense]
    bs = DevBatch(wc, flat)
    bs.forward(wc, ctx)
    ctx.synchronize()
    ctx.set_option(WC_OPT_TICKETS, 0)
    try:
        _force_timeout(wc, ctx, lambda: bs.inverse(ctx))  # may or may not wait: it must not fault either way
        ctx.set_option(WC_OPT_TICKETS, 1)
        bs.inverse(ctx)
        ctx.synchronize()
        got = bs.out.cpu().numpy()
        for i, b in enumerate(flat):
            o = bs.units[i].cell_offset
            want = oracle.decompress_payload(bs.payloads()[i]).ravel()
            assert got[o:o + b.size].tobytes() == want.tobytes(), i
    finally:
        ctx.set_option(WC_OPT_TICKETS, 0)


def test_shared_device_env_selects_tickets():
    code = ("import sys; sys.path.insert(0, %r); import wcamd; from wavelet_compression_amd.capi import "
            "WC_OPT_ORDERED; c = wcamd.capi.Context(0); print('ORDERED', c.get_option(WC_OPT_ORDERED)); "
            "c.close()" % str(ROOT))
    for env_val, want in (("1", 0), ("0", 1)):
        env = dict(os.environ, WCAMD_SHARED_DEVICE=env_val)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=180)
        assert r.returncode == 0, r.stderr[-2000:]
        assert f"ORDERED {want}" in r.stdout, (env_val, r.stdout)
