"""Multi-rank sharding on CPU (gloo, world_size 2): the unit partition, the
metrics all-reduce and that a sharded run reproduces the single-process
payloads.  The per-unit compute here is the CPU oracle (these ranks have no
GPU); the GPU ranks of bench.py use the same plan_shards / reduce_metrics."""
import os
import socket

import numpy as np
import pytest


def test_plan_shards_contiguous_and_balanced(wc):
    from wavelet_compression_amd.shard import plan_shards
    counts = [64 ** 3] * 64 + [32 ** 3] * 96 + [16 ** 3] * 256
    for world in (1, 2, 4, 8):
        sh = plan_shards(counts, world)
        assert sh[0][0] == 0 and sh[-1][1] == len(counts)
        assert all(a[1] == b[0] for a, b in zip(sh, sh[1:]))
        loads = [sum(counts[a:b]) for a, b in sh]
        assert max(loads) - sum(counts) / world <= max(counts)
    assert plan_shards([5], 4) == [(0, 0), (0, 0), (0, 1), (1, 1)] or \
        sum(b - a for a, b in plan_shards([5], 4)) == 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, dims, keep, out_q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WCAMD_NO_TORCH="1")
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import wcamd
    from wavelet_compression_amd.shard import plan_shards, reduce_metrics
    from oracle import oracle as O
    counts = [w * h * d for (w, h, d) in dims]
    a, b = plan_shards(counts, world)[rank]
    payloads, kept = {}, 0
    for u in range(a, b):
        cells = O.synth_box_f64(O.unit_seed(0, 0, u, 0), (0, 0, 0), *dims[u])
        p, k = O.compress_payload(O.narrow(cells), keep)
        payloads[u] = p
        kept += k
    m = reduce_metrics({"cells": sum(counts[a:b]), "kept": kept, "boxes": b - a,
                        "payload_bytes": sum(len(p) for p in payloads.values()),
                        "seconds": 0.1 * (rank + 1), "min_value": float(rank), "max_value": float(rank)})
    gathered = [None] * world
    dist.all_gather_object(gathered, payloads)
    if rank == 0:
        merged = {}
        for g in gathered:
            merged.update(g)
        out_q.put((m, merged))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_reproduce_single_process(wc, oracle):
    import torch.multiprocessing as mp
    dims = [(16, 16, 16), (8, 4, 2), (32, 16, 8), (6, 10, 14), (16, 32, 64), (3, 5, 7)]
    keep = float(np.float32(0.999))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, dims, keep, q)) for r in range(2)]
    for p in procs:
        p.start()
    m, merged = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = {}
    kept = 0
    for u, d in enumerate(dims):
        cells = oracle.synth_box_f64(oracle.unit_seed(0, 0, u, 0), (0, 0, 0), *d)
        p, k = oracle.compress_payload(oracle.narrow(cells), keep)
        single[u] = p
        kept += k
    assert merged == single
    assert m["kept"] == kept and m["boxes"] == len(dims)
    assert m["cells"] == sum(w * h * d for (w, h, d) in dims)
    assert m["seconds"] == pytest.approx(0.2) and m["min_value"] == 0.0 and m["max_value"] == 1.0


class _OracleStageCtx:
    """Stands in for capi.Context on a CPU rank: forward_stage adds the oracle's
    coefficient-magnitude histogram of this rank's units to the hist buffer."""

    def __init__(self, O, units):
        self.O, self.units = O, units

    def forward_stage(self, d_cells, dtype, units, n, d_hist):
        import ctypes
        h = np.ctypeslib.as_array((ctypes.c_uint64 * self.O.HIST_BINS).from_address(d_hist))
        for cells in self.units:
            h += self.O.magnitude_hist(self.O.wavelet_decompose(self.O.narrow(cells)))

    def synchronize(self):
        pass


def _hist_worker(rank, world, port, dims, quantile, out_q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    sys.path.insert(0, str(root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WCAMD_NO_TORCH="1")
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import wcamd  # noqa: F401
    from wavelet_compression_amd.shard import global_threshold, plan_shards
    from oracle import oracle as O
    a, b = plan_shards([w * h * d for (w, h, d) in dims], world)[rank]
    cells = [O.synth_box_f64(O.unit_seed(0, 0, u, 0), (0, 0, 0), *dims[u]) for u in range(a, b)]
    hist = torch.zeros(O.HIST_BINS, dtype=torch.int64)
    thresh, retained = global_threshold(_OracleStageCtx(O, cells), 0, 1, None, b - a, quantile, hist)
    payloads = {u: O.compress_payload_thresh(O.narrow(c), thresh) for u, c in zip(range(a, b), cells)}
    gathered = [None] * world
    dist.all_gather_object(gathered, (thresh, retained, payloads))
    if rank == 0:
        out_q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("quantile", [0.5, 0.9])
def test_gloo_global_histogram_threshold(wc, oracle, quantile):
    """Opt-in global-threshold mode over two gloo ranks: one all-reduce of the
    4096-bin histogram gives every rank the threshold a single process computes
    over all units, and the kept count equals the histogram's retained count."""
    import torch.multiprocessing as mp
    dims = [(16, 16, 16), (8, 4, 2), (32, 16, 8), (6, 10, 14), (16, 32, 64), (3, 5, 7)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hist_worker, args=(r, 2, port, dims, quantile, q)) for r in range(2)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    flats = [oracle.wavelet_decompose(oracle.narrow(
        oracle.synth_box_f64(oracle.unit_seed(0, 0, u, 0), (0, 0, 0), *d))) for u, d in enumerate(dims)]
    hist = sum(oracle.magnitude_hist(f) for f in flats)
    thresh, retained = oracle.hist_threshold(hist, quantile)
    assert wc.capi.hist_threshold(hist, quantile) == (thresh, retained)
    merged = {}
    for t, r, p in gathered:
        assert (t, r) == (thresh, retained)
        merged.update(p)
    total = sum(int(f.size) for f in flats)
    kept = sum(int(np.count_nonzero(np.abs(f.astype(np.float64)) > thresh)) for f in flats)
    assert kept == retained >= total - int(np.floor(quantile * total))
    assert merged == {u: oracle.compress_payload_thresh(oracle.narrow(
        oracle.synth_box_f64(oracle.unit_seed(0, 0, u, 0), (0, 0, 0), *d)), thresh) for u, d in enumerate(dims)}


def test_bench_spawns_ranks_and_merges_one_line(tmp_path):
    """bench.py --gpus 2 (no WORLD_SIZE in the environment) starts two ranks
    itself (torch.distributed.run), shards C5 / C4 over them with plan_shards
    and prints ONE merged JSON line from rank 0 (gloo on CPU: --plumbing runs
    the launcher, shards and reductions without kernels)."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["WCAMD_NO_TORCH"] = "1"
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--plumbing"], env=env,
                       capture_output=True, text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["ranks_seen"] == 2
    assert out["max_seconds"] == pytest.approx(0.002)
    for name, sh in out["shards"].items():
        assert sh["cells_total"] == sh["expected_total"], name
        assert sh["rank0_span"][0] == 0 and 0 < sh["rank0_span"][1] < sh["units_total"], name


def test_bench_force_dist_takes_the_process_group_path_at_world1(tmp_path):
    """bench.py --force-dist at one rank: started through torch.distributed.run
    (no WORLD_SIZE in the environment), the Dist process-group path with every
    reduction a real collective (gloo here; RCCL on the GPU box,
    test_gpu_rccl.py), one line naming the backend."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["WCAMD_NO_TORCH"] = "1"
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--force-dist", "--plumbing"], env=env,
                       capture_output=True, text=True, timeout=300, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["ranks_seen"] == 1 and out["dist_backend"] == "gloo"
    for name, sh in out["shards"].items():
        assert sh["cells_total"] == sh["expected_total"], name


def test_bench_rank_failure_ends_the_job_fast(tmp_path):
    """One rank of `bench.py --gpus 2` raises before the first collective: the
    launcher exits non-zero well within the process-group timeout and leaves
    no rank waiting (torch.distributed.run stops the other rank; its own
    collectives are bounded by --dist-timeout besides)."""
    import subprocess
    import sys
    import time
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["WCAMD_NO_TORCH"] = "1"
    for fail in (1, 0):
        t0 = time.monotonic()
        p = subprocess.Popen([sys.executable, str(root / "bench.py"), "--gpus", "2", "--plumbing",
                              "--fail-rank", str(fail), "--dist-timeout", "30"], env=env, cwd=tmp_path,
                             stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
        try:
            out, err = p.communicate(timeout=120)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, 9)
            raise AssertionError(f"rank {fail} failing left the job hanging")
        took = time.monotonic() - t0
        assert p.returncode != 0, out
        assert "injected failure" in err, err[-2000:]
        assert not [ln for ln in out.splitlines() if ln.startswith("{")], out
        assert took < 90, took
        # no process of the job is left behind (its session is empty)
        r = subprocess.run(["pgrep", "-s", str(p.pid)], capture_output=True, text=True)
        assert r.stdout.strip() == "", r.stdout


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu(tmp_path):
    """The driver's multi-GPU bench path on a one-GPU box: `bench.py --gpus 2
    --rehearse` starts two ranks (gloo, both on device 0) that run the real
    kernels on their own shards (C5 split by plan_shards) and merge ONE line
    whose totals cover both ranks."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--rehearse", "--steps", "2",
                        "--warmup", "1", "--leg-steps", "1", "--legs", "c5", "--no-cpu-baseline"], env=env,
                       capture_output=True, text=True, timeout=240, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 2048
    assert out["value"] > 0 and 0.25 < out["kept_fraction"] < 0.35
    c5 = out["c5"]
    assert c5["units_total"] == 512 and c5["units_this_rank"] == 256 and c5["cells_total"] == 512 * 128 ** 3
    # both ranks' kept totals add up to the line's, at C5's density (keep 0.9999f on 128^3)
    pr = c5["per_rank"]
    assert len(pr) == 2 and [p["units"] for p in pr] == [256, 256]
    assert sum(p["kept"] for p in pr) == round(c5["kept_fraction"] * c5["cells_total"])
    for p in pr:
        assert 0.35 < p["kept"] / p["cells"] < 0.55, p
    # each rank's first 128^3 unit: its payload bytes are the oracle's
    import hashlib

    import numpy as np
    import torch
    import bench_workloads as bw
    from oracle import oracle as O
    units = bw.WORKLOADS["c5"]["units"]()
    assert [p["first_unit"]["unit"] for p in pr] == [0, 256]
    for p in pr:
        u = units[p["first_unit"]["unit"]]
        cells, _, _ = bw.synth_cells(torch, torch.device("cuda", 0), [u], "f32")
        box = cells[:u.cells].cpu().numpy().reshape(u.D, u.H, u.W)
        want, wk = O.compress_payload(box, float(np.float32(0.9999)))
        assert p["first_unit"]["kept"] == wk
        assert p["first_unit"]["sha256"] == hashlib.sha256(want).hexdigest(), p
