"""bench.py — the forward hot path (transform + keep threshold + ordered pack)
of the wavelet codec on MI355X, plus the inverse / round-trip legs of the
other BASELINE.json configs.

Headline (`value`, BASELINE.json configs[1] = C2): 1024 synthetic 64^3 fp64
boxes per GPU, 1 component, keep = 0.999f, inputs resident in HBM before the
timed region; one step = one wc_forward over the rank's whole batch (cells ->
serialized payloads, byte-identical to the reference's serialize()).  N GPUs:
one process per GPU, each compressing its own 1024 boxes (independent AMR
units, no data-path collective) -> weak scaling; `value` = all ranks' cells /
the slowest rank's time.

Legs (sub-objects of the same JSON line):
  inverse  C2's payloads back to cells (rle_decode + inverse transform) and
           the per-box RMSE (calc_rmse_per_box) of the reconstruction
  host     C2 through the host-buffer boundary (wc_forward_host: pinned host
           cells over PCIe, packed payloads back to host memory): the
           PCIe-inclusive rate, reported beside `value`, never as it
  c3       BASELINE configs[2]: 4-level AMR layout x 4 components, fwd + inv +
           RMSE round trip on one GPU (world == 1)
  c5       configs[4]: 512 x 128^3 fp32, keep 0.9999, units split over ranks
  c4       configs[3]: 10 timesteps x 4 levels x 8 components, units split over
           ranks; plus the opt-in global-threshold mode (magnitude histogram,
           ONE all-reduce over ranks: RCCL over xGMI)
  cpu_baseline  (rank 0, world 1) the CPU restatement on the host cores on a
           bounded sample, with and without xz preset 6; sample parity and the
           RMSE check against it.

`python bench.py --gpus N` without WORLD_SIZE in the environment starts N
ranks itself (torch.distributed.run, before any GPU call); under an outer
torchrun it is one rank.  `--plumbing` runs the rank/shard/reduction logic on
CPU (gloo) without kernels, for the CPU test suite.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
ALL_LEGS = ("inverse", "host", "f32_64", "c3", "c5", "c4")
OPT_LEGS = ("cli", "dropin")  # opt-in (--legs ...): subprocess runs of the CLI and of the drop-in driver


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("c2", "c3", "c4", "c5", "f32_64"), default="c2",
                    help="headline workload (default: BASELINE configs[1], C2)")
    ap.add_argument("--legs", default=",".join(ALL_LEGS),
                    help="comma list of extra legs (inverse,host,f32_64,c3,c5,c4; opt-in: cli,dropin) or 'none'")
    ap.add_argument("--leg-steps", type=int, default=5, help="timed steps of each extra leg")
    ap.add_argument("--hist-quantile", type=float, default=0.7,
                    help="c4 leg: quantile of the opt-in global-threshold mode (NOT the reference rule)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="time budget of each CPU-baseline sample (boxes run until it is spent)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default=str(ROOT / "profiles" / "r06"),
                    help="PMC traffic summaries (tools/pmc_summary.py): a file or a directory of pmc_*.json, "
                         "one per workload; merged into roofline.traffic and each leg's roofline_path.traffic "
                         "when measured on the same workload AND the same kernel sources")
    ap.add_argument("--rix-xcd", action="store_true",
                    help="diagnostic: row-indexed inverse tiles in XCD-grouped order (WC_OPT_RIX_XCD 1)")
    ap.add_argument("--inv-groups", type=int, default=0,
                    help="diagnostic: WC_OPT_INV_GROUPS of the inverse legs (0: the library default)")
    ap.add_argument("--dist-timeout", type=float, default=120.0,
                    help="seconds a rank waits at process-group setup or in a collective before failing "
                         "(a rank that died leaves the others failing fast instead of hanging)")
    ap.add_argument("--fail-rank", type=int, default=-1,
                    help="test hook (--plumbing only): this rank raises before its first collective")
    ap.add_argument("--plumbing", action="store_true",
                    help="CPU/gloo run of the launcher, sharding and reductions (no kernels, no numbers)")
    ap.add_argument("--force-dist", action="store_true",
                    help="take the process-group path even at one rank (RCCL at world 1 on a one-GPU box: "
                         "init, barriers, metric reductions, all_gather_object and the histogram all-reduce "
                         "run over the real backend)")
    ap.add_argument("--rehearse", action="store_true",
                    help="multi-rank rehearsal on a one-GPU box: every rank on device 0, gloo instead of RCCL "
                         "(the kernels, shards and reductions of --gpus N; the numbers are not a scaling result)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """Start `--gpus` ranks with torch.distributed.run (one process per GPU) and
    return its exit status.  Called before anything touches the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve())]
    cmd += sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------
# helpers

def kernel_sources_sha() -> str:
    """Hash of the kernel + C-ABI sources: a PMC summary applies only to them."""
    h = hashlib.sha256()
    cs = ROOT / "wavelet-compression_amd" / "csrc"
    for p in sorted(list(cs.glob("*.hip")) + list(cs.glob("*.h")) + list(cs.glob("wc_*.cpp"))):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def alg_bytes_forward(s_in, cells, kept, nunits):
    """B = s_in*N_cells + 8*N_kept + 20*N_units."""
    return s_in * cells + 8 * kept + 20 * nunits


def alg_bytes_inverse(cells, kept, nunits):
    """B = 8*N_kept + 20*N_units + 4*N_cells."""
    return 8 * kept + 20 * nunits + 4 * cells


class Dist:
    """The rank's view of the job: world, rank, device, barrier, reductions."""

    def __init__(self, plumbing: bool, rehearse: bool = False, timeout_s: float = 120.0, force: bool = False):
        import datetime

        import torch
        import torch.distributed as dist
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.plumbing = plumbing
        # collectives run whenever there is a process group: world > 1, or
        # --force-dist at world 1 (the backend exercised on a one-GPU box)
        self.distributed = self.world > 1 or force
        self.coll_dev = None  # device of the reduction tensors (None: self.dev)
        # bounded setup and collectives: a rank that died before a collective
        # makes the others fail after this long (torch.distributed.run also
        # stops the remaining ranks as soon as one exits non-zero)
        tmo = datetime.timedelta(seconds=timeout_s)
        if plumbing:
            self.dev = torch.device("cpu")
            if self.distributed:
                dist.init_process_group("gloo", timeout=tmo)
        elif rehearse:
            if self.distributed:
                dist.init_process_group("gloo", timeout=tmo)
            torch.cuda.set_device(0)
            self.dev = torch.device("cuda", 0)
            self.local = 0
            self.coll_dev = torch.device("cpu")
        else:
            if self.distributed:
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local), timeout=tmo)
            torch.cuda.set_device(self.local)
            self.dev = torch.device("cuda", self.local)

    def backend(self):
        if not self.distributed:
            return None
        import torch.distributed as dist
        b = dist.get_backend()
        return "RCCL over xGMI" if b == "nccl" else b

    def barrier(self):
        if self.distributed:
            import torch.distributed as dist
            dist.barrier()

    def reduce(self, metrics):
        if not self.distributed:
            return dict(metrics)
        from wavelet_compression_amd.shard import reduce_metrics
        return reduce_metrics(metrics, device=self.coll_dev or self.dev)

    def gather(self, obj):
        """Every rank's `obj` (a small JSON-able value), in rank order."""
        if not self.distributed:
            return [obj]
        import torch.distributed as dist
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.distributed:
            import torch.distributed as dist
            dist.destroy_process_group()


def rank_units(name, d: Dist):
    """This rank's units of a workload: its own copy (per-GPU workloads, unit
    ids offset by rank) or its contiguous cell-balanced share (shard.plan_shards)."""
    import bench_workloads as bw
    from wavelet_compression_amd.shard import plan_shards
    spec = bw.WORKLOADS[name]
    units = spec["units"]()
    if spec["per_gpu"]:
        n = len(units)
        return [bw.Unit(u.t, u.lev, u.box, u.comp, u.W, u.H, u.D,
                        (u.lo[0], u.lo[1], u.lo[2] + 4096 * d.rank), u.gid + n * d.rank) for u in units], (0, n)
    a, b = plan_shards([u.cells for u in units], d.world)[d.rank]
    return units[a:b], (a, b)


class Batch:
    """A rank's batch on the device: cells, the unit table and output buffers."""

    def __init__(self, d: Dist, units, dtype, keep, inverse=False):
        import numpy as np
        import torch
        import bench_workloads as bw
        import wcamd
        self.capi = wcamd.capi
        self.units = units
        self.dtype = dtype
        self.keep = float(np.float32(keep))  # Config::keep is a float (src/argparse.h:13)
        self.s_in = 8 if dtype == "f64" else 4
        self.code = self.capi.WC_F64 if dtype == "f64" else self.capi.WC_F32
        self.cells_dev, offs, self.extent = bw.synth_cells(torch, d.dev, units, dtype)
        self.tab, self.n, _ = bw.units_array(self.capi, units, offs)
        self.offs = offs
        self.ncells = sum(u.cells for u in units)
        self.cap = self.capi.payload_bound(self.tab, self.n) if self.n else 16
        self.payload = torch.empty(self.cap, dtype=torch.uint8, device=d.dev)
        self.offsets = torch.zeros(self.n + 1, dtype=torch.int64, device=d.dev)
        self.kept = torch.zeros(max(self.n, 1), dtype=torch.int32, device=d.dev)
        self.regen = torch.empty(max(self.extent, 1), dtype=torch.float32, device=d.dev) if inverse else None
        self.rmse = torch.zeros(max(self.n, 1), dtype=torch.float64, device=d.dev) if inverse else None
        # the payloads' row index (wc_forward_rows / wc_inverse_rows: in-process round trips)
        self.rows_bytes = self.capi.rowindex_bytes(self.tab, self.n) if (inverse and self.n) else 0
        self.rows = torch.empty(max(self.rows_bytes // 8, 1), dtype=torch.int64, device=d.dev) if inverse else None
        torch.cuda.synchronize()

    def forward(self, ctx):
        if self.n:
            ctx.forward(self.cells_dev.data_ptr(), self.code, self.tab, self.n, self.keep, self.payload.data_ptr(),
                        self.cap, self.offsets.data_ptr(), self.kept.data_ptr())

    def inverse(self, ctx):
        if self.n:
            ctx.inverse(self.payload.data_ptr(), self.offsets.data_ptr(), self.tab, self.n, self.regen.data_ptr())

    def rmse_step(self, ctx):
        if self.n:
            ctx.rmse(self.cells_dev.data_ptr(), self.code, self.regen.data_ptr(), self.tab, self.n,
                     self.rmse.data_ptr())

    def inverse_rmse(self, ctx):
        if self.n:
            ctx.inverse_rmse(self.payload.data_ptr(), self.offsets.data_ptr(), self.tab, self.n,
                             self.cells_dev.data_ptr(), self.code, self.regen.data_ptr(), self.rmse.data_ptr())

    def forward_rows(self, ctx):
        if self.n:
            ctx.forward_rows(self.cells_dev.data_ptr(), self.code, self.tab, self.n, self.keep,
                             self.payload.data_ptr(), self.cap, self.offsets.data_ptr(), self.kept.data_ptr(),
                             self.rows.data_ptr(), self.rows_bytes)

    def inverse_rows(self, ctx):
        if self.n:
            ctx.inverse_rows(self.payload.data_ptr(), self.offsets.data_ptr(), self.tab, self.n,
                             self.rows.data_ptr(), self.regen.data_ptr())

    def inverse_rows_rmse(self, ctx):
        if self.n:
            ctx.inverse_rows(self.payload.data_ptr(), self.offsets.data_ptr(), self.tab, self.n,
                             self.rows.data_ptr(), self.regen.data_ptr(), self.cells_dev.data_ptr(), self.code,
                             self.rmse.data_ptr())

    def kept_total(self):
        return int(self.kept[:self.n].to(self.kept.device).sum().item()) if self.n else 0


def new_context(args, d: Dist):
    """The rank's library context (the default launch-order look-backs, also
    for ranks sharing one GPU under --rehearse: no wait depends on which
    process's workgroups are dispatched, DESIGN.md §Forward progress)."""
    import wcamd
    ctx = wcamd.capi.Context(d.local)
    if args.rix_xcd:
        ctx.set_option(wcamd.capi.WC_OPT_RIX_XCD, 1)
    if args.inv_groups:
        ctx.set_option(wcamd.capi.WC_OPT_INV_GROUPS, args.inv_groups)
    return ctx


def timed(d: Dist, ctx, step, steps, warmup):
    """Warmup, then EXACTLY `steps` steps bracketed by barrier + synchronize on
    both sides; returns this rank's seconds.  No per-kernel events inside."""
    import torch
    for _ in range(warmup):
        step()
    ctx.synchronize()
    d.barrier()
    torch.cuda.synchronize()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    d.barrier()
    return time.perf_counter() - t0


def stage_times(ctx, step, steps):
    """Per-kernel average launch times (ms) from hipEvents recorded on the
    context stream around each launch, from `steps` more steps."""
    ctx.profile_enable(True)
    ctx.profile_read()
    for _ in range(steps):
        step()
    ctx.synchronize()
    ctx.profile_enable(False)
    return {k: (ms / cnt, cnt / steps) for k, (ms, cnt) in ctx.profile_read().items()}


FWD_STAGES = ("transform", "fallback", "emit")
HIST_STAGES = ("transform", "hist", "emit")
INV_STAGES = ("rowindex", "decode", "inverse", "rmse", "pairs")


def pmc_summary(path, workload, dtype):
    """The committed rocprofv3 PMC summary of `workload` (a file, or pmc_*.json in a
    directory), only if measured on this workload AND these kernel sources."""
    p = Path(path)
    files = sorted(p.glob("pmc_*.json")) if p.is_dir() else ([p] if p.exists() else [])
    meta = {"source": None, "note": "no PMC summary for this workload"}
    for f in files:
        try:
            pmc = json.loads(f.read_text())
        except Exception:
            continue
        cfg = pmc.get("config", {})
        if cfg.get("workload") != workload or cfg.get("dtype") != dtype:
            continue
        meta = {"source": str(f.relative_to(ROOT)) if f.is_relative_to(ROOT) else str(f),
                "date": pmc.get("date"), "git": pmc.get("git")}
        if pmc.get("kernel_sources_sha") != kernel_sources_sha():
            meta["note"] = "stale: kernel sources changed since the counter run"
            return None, meta
        return pmc, meta
    return None, meta


def pmc_traffic(path, workload, dtype, kernel):
    """Counter bytes per launch of `kernel` (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE)."""
    pmc, meta = pmc_summary(path, workload, dtype)
    return (pmc.get("per_launch_bytes", {}).get(kernel) if pmc else None), meta


def path_traffic(path, workload, dtype, stages, alg_bytes):
    """Counter bytes per step of the kernels of `stages`, beside the algorithmic bytes."""
    pmc, meta = pmc_summary(path, workload, dtype)
    per = (pmc or {}).get("per_step_bytes")
    if not per:
        return {"traffic": None, "traffic_source": meta}
    t = sum(v for k, v in per.items() if k in stages)
    return {"traffic": t, "traffic_ratio": t / alg_bytes if alg_bytes else None,
            "traffic_by_kernel": {k: v for k, v in per.items() if k in stages}, "traffic_source": meta}


# ---------------------------------------------------------------------------
# the headline workload

def headline(args, d: Dist, ctx):
    import bench_workloads as bw
    spec = bw.WORKLOADS[args.workload]
    units, span = rank_units(args.workload, d)
    b = Batch(d, units, spec["dtype"], spec["keep"], inverse="inverse" in args.legs_set)
    secs = timed(d, ctx, lambda: b.forward(ctx), args.steps, args.warmup)
    stages = stage_times(ctx, lambda: b.forward(ctx), args.steps)
    kept = b.kept_total()
    m = d.reduce({"seconds": secs, "kept": kept, "cells": b.ncells, "boxes": b.n,
                  "payload_bytes": 8 * kept + 20 * b.n})
    elapsed = m["seconds"]
    # roofline of the dominant kernel: its algorithmic bytes per launch / its launch time
    own = {"transform": b.s_in * b.ncells, "emit": 8 * kept + 20 * b.n}
    dominant = max(stages, key=lambda k: stages[k][0])
    dom_ms = stages[dominant][0]
    achieved = own.get(dominant, 0) / (dom_ms * 1e-3) / 1e9
    path_ms = sum(v[0] * v[1] for v in stages.values())
    path_bytes = alg_bytes_forward(b.s_in, b.ncells, kept, b.n)
    traffic, tmeta = pmc_traffic(args.pmc, args.workload, spec["dtype"], dominant)
    ms_step = elapsed / args.steps * 1e3
    out = {
        "metric": f"{'fp64' if spec['dtype'] == 'f64' else 'fp32'} cells/s, fwd transform+threshold+pack, "
                  f"keep={spec['keep']}",
        "value": m["cells"] * args.steps / elapsed,
        "unit": "cells/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak" if spec["per_gpu"] else "strong",
        "vs_baseline": None,
        "dtype": spec["dtype"],
        "data": "synthetic (SURVEY §8(d) field + N(0,0.05) noise, generated on device; bench_workloads.py)",
        "dist_backend": d.backend(),
        "config": {"workload": f"{args.workload}: {spec['desc']}, wc_forward (payload bytes identical to the "
                               f"reference's serialize())",
                   "boxes_per_gpu": b.n, "global_batch": int(m["boxes"]),
                   "parallelism": f"box-sharded x{d.world}"},
        "compressed_GBps": m["cells"] * b.s_in * args.steps / elapsed / 1e9,
        "kept_fraction": m["kept"] / max(m["cells"], 1),
        "payload_bytes_per_step": int(m["payload_bytes"]),
        "stage_ms_per_launch": {k: round(v[0], 4) for k, v in stages.items()},
        "roofline": {
            "bound": "hbm", "kernel": dominant,
            "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBPS,
            "traffic": traffic,
            "traffic_GBps": (traffic / (dom_ms * 1e-3) / 1e9) if traffic else None,
            "traffic_source": tmeta,
            "alg_bytes_per_launch": own.get(dominant, 0),
        },
        "roofline_path": {"achieved": path_bytes / (ms_step * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS,
                          "unit": "GB/s", "frac": path_bytes / (ms_step * 1e-3) / 1e9 / PEAK_HBM_GBPS,
                          "bytes_per_step": path_bytes, "kernel_ms_per_step": path_ms,
                          "note": "algorithmic bytes / driver-clock ms_per_step (launch gaps included)",
                          **path_traffic(args.pmc, args.workload, spec["dtype"], FWD_STAGES, path_bytes)},
    }
    return out, b


def inverse_leg(args, d: Dist, ctx, b: Batch):
    """C2's payloads back to cells + per-box RMSE; SURVEY §8(d) inverse bytes."""
    import torch
    kept = b.kept_total()
    secs = timed(d, ctx, lambda: b.inverse(ctx), args.steps, 2)
    st = stage_times(ctx, lambda: b.inverse(ctx), args.steps)
    b.rmse_step(ctx)
    ctx.synchronize()
    r = b.rmse[:b.n]
    m = d.reduce({"seconds": secs, "cells": b.ncells, "kept": kept, "boxes": b.n,
                  "rmse_sum": float(r.sum().item()), "max_rmse": float(r.max().item())})
    ms = m["seconds"] / args.steps * 1e3
    alg = alg_bytes_inverse(b.ncells, kept, b.n)
    # the in-process round trip's inverse: the same payloads with the row index
    # wc_forward_rows wrote beside them (wc_inverse_rows: no row index kernel)
    b.forward_rows(ctx)
    ctx.synchronize()
    rsecs = timed(d, ctx, lambda: b.inverse_rows(ctx), args.steps, 2)
    rst = stage_times(ctx, lambda: b.inverse_rows(ctx), args.steps)
    rms = d.reduce({"seconds": rsecs})["seconds"] / args.steps * 1e3
    torch.cuda.synchronize()
    return {"value": m["cells"] / (ms * 1e-3), "unit": "cells/s", "ms_per_step": ms,
            "with_forward_row_index": {
                "ms_per_step": rms, "value": m["cells"] / (rms * 1e-3), "unit": "cells/s",
                "stage_ms_per_launch": {k: round(v[0], 4) for k, v in rst.items()},
                "roofline_path": {"achieved": alg / (rms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                                  "frac": alg / (rms * 1e-3) / 1e9 / PEAK_HBM_GBPS},
                "note": "wc_inverse_rows of the same payloads with the row index wc_forward_rows wrote "
                        "(the -estimate / round-trip form; `ms_per_step` above: wc_inverse from the payloads "
                        "alone, the -d form)"},
            "stage_ms_per_launch": {k: round(v[0], 4) for k, v in st.items()},
            "roofline_path": {"achieved": alg / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                              "frac": alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, "bytes_per_step": alg,
                              **path_traffic(args.pmc, args.workload, "f64" if b.s_in == 8 else "f32",
                                             INV_STAGES, alg)},
            "rmse": {"mean_per_box": m["rmse_sum"] / max(m["boxes"], 1), "max": m["max_rmse"],
                     "note": "calc_rmse_per_box of the reconstruction vs the narrowed input (GPU K7); "
                             "checked against the CPU restatement in cpu_baseline.rmse_check"}}


def round_trip_leg(args, d: Dist, name):
    """C3: forward + inverse + RMSE per step over the whole AMR layout (one GPU)."""
    import bench_workloads as bw
    import torch
    import wcamd
    spec = bw.WORKLOADS[name]
    units, _ = rank_units(name, d)
    ctx = new_context(args, d)
    b = Batch(d, units, spec["dtype"], spec["keep"], inverse=True)

    def separate():
        b.forward(ctx)
        b.inverse(ctx)
        b.rmse_step(ctx)

    def fused():  # wc_inverse_rmse: the RMSE fused into the row-indexed inverse, the row index from the payloads
        b.forward(ctx)
        b.inverse_rmse(ctx)

    def step():  # the forward writes the row index, the inverse reads it (no row index kernel)
        b.forward_rows(ctx)
        b.inverse_rows_rmse(ctx)

    sep_ms = timed(d, ctx, separate, args.leg_steps, 2) / args.leg_steps * 1e3
    fused_ms = timed(d, ctx, fused, args.leg_steps, 2) / args.leg_steps * 1e3
    secs = timed(d, ctx, step, args.leg_steps, 2)
    st = stage_times(ctx, step, args.leg_steps)
    kept = b.kept_total()
    r = b.rmse[:b.n].cpu().numpy()
    ms = secs / args.leg_steps * 1e3
    fwd = alg_bytes_forward(b.s_in, b.ncells, kept, b.n)
    inv = alg_bytes_inverse(b.ncells, kept, b.n)
    rm = b.s_in * b.ncells  # fused: the original cells (the reconstruction is not re-read)
    per_comp = {}
    for u, v in zip(units, r):
        per_comp.setdefault(u.comp, []).append(float(v))
    out = {"workload": spec["desc"], "units": b.n, "cells": b.ncells, "dtype": spec["dtype"],
           "kept_fraction": kept / b.ncells, "ms_per_step": ms,
           "round_trip_cells_per_s": b.ncells / (ms * 1e-3),
           "path": "wc_forward_rows + wc_inverse_rows (fused RMSE, the forward's row index)",
           "fused_from_payload_ms_per_step": fused_ms,
           "separate_calls_ms_per_step": sep_ms,
           "stage_ms_per_step": {k: round(v[0] * v[1], 4) for k, v in st.items()},
           "roofline_path": {"bytes_per_step": fwd + inv + rm, "achieved": (fwd + inv + rm) / (ms * 1e-3) / 1e9,
                             "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                             "frac": (fwd + inv + rm) / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS,
                             "note": "fwd + inverse + RMSE algorithmic bytes (RMSE: original cells only, "
                                     "fused) / driver-clock step",
                             **path_traffic(args.pmc, name, spec["dtype"], FWD_STAGES + INV_STAGES,
                                            fwd + inv + rm)},
           "mean_rmse_per_component": {str(c): sum(v) / len(v) for c, v in sorted(per_comp.items())}}
    ctx.close()
    del b
    torch.cuda.empty_cache()
    return out


def sharded_forward_leg(args, d: Dist, name, hist=False, inverse=False):
    """C5 / C4: the workload's units split over ranks (plan_shards), forward timed
    as the headline; C4 adds the opt-in global-threshold mode (one all-reduce).
    f32_64: C2's shape in fp32 per GPU (weak).  inverse: also wc_inverse of the
    leg's payloads (rle_decode + inverse transform, src/decompressor.cpp:238-255)."""
    import bench_workloads as bw
    import torch
    import wcamd
    spec = bw.WORKLOADS[name]
    units, span = rank_units(name, d)
    ctx = new_context(args, d)
    b = Batch(d, units, spec["dtype"], spec["keep"], inverse=inverse)
    secs = timed(d, ctx, lambda: b.forward(ctx), args.leg_steps, 2)
    st = stage_times(ctx, lambda: b.forward(ctx), args.leg_steps)
    kept = b.kept_total()
    m = d.reduce({"seconds": secs, "cells": b.ncells, "kept": kept, "boxes": b.n,
                  "max_rank_cells": b.ncells, "min_rank_cells": b.ncells})
    ms = m["seconds"] / args.leg_steps * 1e3
    alg = alg_bytes_forward(b.s_in, m["cells"], m["kept"], m["boxes"])
    per_rank_alg = alg_bytes_forward(b.s_in, b.ncells, kept, b.n)
    # per rank: its kept total and the digest of its first unit's payload (the
    # GPU test recomputes that unit with the oracle; bench.py itself checks nothing)
    sample = None
    if b.n:
        o, k = int(b.offsets[0].item()), int(b.kept[0].item())
        sample = {"unit": units[0].gid, "kept": k,
                  "sha256": hashlib.sha256(b.payload[o:o + 20 + 8 * k].cpu().numpy().tobytes()).hexdigest()}
    per_rank = d.gather({"kept": kept, "cells": b.ncells, "units": b.n, "first_unit": sample})
    out = {"workload": spec["desc"], "units_total": int(m["boxes"]), "units_this_rank": b.n,
           "rank0_span": list(span), "cells_total": int(m["cells"]), "dtype": spec["dtype"], "keep": spec["keep"],
           "kept_fraction": m["kept"] / max(m["cells"], 1), "ms_per_step": ms,
           "value": m["cells"] / (ms * 1e-3), "unit": "cells/s", "scaling": "weak" if spec["per_gpu"] else "strong",
           "rank_cell_balance": m["max_rank_cells"] / max(m["min_rank_cells"], 1),
           "per_rank": per_rank,
           "stage_ms_per_launch": {k: round(v[0], 4) for k, v in st.items()},
           "roofline_path": {"achieved_per_gpu": per_rank_alg / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS,
                             "unit": "GB/s", "frac": per_rank_alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS,
                             "bytes_per_step_all_ranks": alg,
                             **(path_traffic(args.pmc, name, spec["dtype"], FWD_STAGES, per_rank_alg)
                                if d.world == 1 else {"traffic": None, "traffic_source": {
                                    "note": "counter summaries are for the one-GPU workload"}})}}
    if hist:
        out["global_hist"] = global_hist_leg(args, d, ctx, b)
    if inverse:
        out["inverse"] = sharded_inverse(args, d, ctx, b, name)
    ctx.close()
    del b
    torch.cuda.empty_cache()
    return out


def sharded_inverse(args, d: Dist, ctx, b: Batch, name):
    """wc_inverse of a leg's payloads, timed as the forward; SURVEY §8(d) inverse
    bytes per rank; counter traffic from the workload's PMC summary (one GPU)."""
    kept = b.kept_total()
    secs = timed(d, ctx, lambda: b.inverse(ctx), args.leg_steps, 2)
    st = stage_times(ctx, lambda: b.inverse(ctx), args.leg_steps)
    m = d.reduce({"seconds": secs, "cells": b.ncells})
    ms = m["seconds"] / args.leg_steps * 1e3
    alg = alg_bytes_inverse(b.ncells, kept, b.n)
    # the in-process round trip's inverse (wc_inverse_rows with the row index
    # wc_forward_rows wrote): no row index kernel
    b.forward_rows(ctx)
    ctx.synchronize()
    rsecs = timed(d, ctx, lambda: b.inverse_rows(ctx), args.leg_steps, 2)
    rst = stage_times(ctx, lambda: b.inverse_rows(ctx), args.leg_steps)
    rms = d.reduce({"seconds": rsecs})["seconds"] / args.leg_steps * 1e3
    return {"value": m["cells"] / (ms * 1e-3), "unit": "cells/s", "ms_per_step": ms,
            "with_forward_row_index": {
                "ms_per_step": rms, "value": m["cells"] / (rms * 1e-3), "unit": "cells/s",
                "stage_ms_per_launch": {k: round(v[0], 4) for k, v in rst.items()},
                "roofline_path": {"achieved_per_gpu": alg / (rms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS,
                                  "unit": "GB/s", "frac": alg / (rms * 1e-3) / 1e9 / PEAK_HBM_GBPS},
                "note": "wc_inverse_rows of the same payloads with the forward's row index (the round-trip "
                        "form; `ms_per_step` above: wc_inverse from the payloads alone, the -d form)"},
            "stage_ms_per_launch": {k: round(v[0], 4) for k, v in st.items()},
            "roofline_path": {"achieved_per_gpu": alg / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                              "frac": alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, "bytes_per_step": alg,
                              **(path_traffic(args.pmc, name, "f64" if b.s_in == 8 else "f32", INV_STAGES, alg)
                                 if d.world == 1 else {"traffic": None, "traffic_source": {
                                     "note": "counter summaries are for the one-GPU workload"}})}}


def global_hist_leg(args, d: Dist, ctx, b: Batch):
    """Opt-in global-threshold mode, timed like a step: stage (K1 + histogram),
    ONE all-reduce of the 4096-bin histogram over all ranks (RCCL over xGMI when
    world > 1), the threshold on the host, one emit."""
    import torch
    from wavelet_compression_amd.shard import global_threshold
    hist = torch.zeros(b.capi.HIST_BINS, dtype=torch.int64, device=d.dev)
    res = {}

    def step():
        hist.zero_()
        t, r = global_threshold(ctx, b.cells_dev.data_ptr(), b.code, b.tab, b.n, args.hist_quantile, hist)
        ctx.forward_emit(b.tab, b.n, 0.0, t, b.payload.data_ptr(), b.cap, b.offsets.data_ptr(),
                         b.kept.data_ptr())
        res.update(thresh=t, retained=r)

    secs = timed(d, ctx, step, args.leg_steps, 1)
    st = stage_times(ctx, step, args.leg_steps)
    kept = b.kept_total()
    m = d.reduce({"seconds": secs, "kept": kept, "cells": b.ncells})
    ms = m["seconds"] / args.leg_steps * 1e3
    # algorithmic bytes: the forward's; the 32 KiB histogram and its all-reduce are noise
    alg = alg_bytes_forward(b.s_in, b.ncells, kept, b.n)
    return {"mode": "global histogram threshold (opt-in, not the reference rule)",
            "quantile": args.hist_quantile, "threshold": res["thresh"], "retained": res["retained"],
            "kept_check": int(m["kept"]) == res["retained"], "kept_fraction": m["kept"] / m["cells"],
            "value": m["cells"] / (ms * 1e-3), "unit": "cells/s", "ms_per_step": ms,
            "stage_ms_per_launch": {k: round(v[0], 4) for k, v in st.items()},
            "roofline_path": {"achieved_per_gpu": alg / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                              "frac": alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, "bytes_per_step": alg,
                              "note": "forward algorithmic bytes / driver-clock step (stage with the histogram folded "
                                      "into K1, host threshold, emit)",
                              **(path_traffic(args.pmc, "c4_hist", "f64" if b.s_in == 8 else "f32", HIST_STAGES, alg)
                                 if d.world == 1 else {"traffic": None, "traffic_source": {
                                     "note": "counter summaries are for the one-GPU workload"}})},
            "allreduce": f"{b.capi.HIST_BINS} x u64 over {d.world} rank(s) ({d.backend() or 'none'})"}


def link_ms(up: int, down: int) -> float:
    """The PCIe floor of a call moving `up` and `down` bytes: each direction
    at most 57 GB/s, both together at most 74.5 GB/s (measured on the MI355X
    boxes, profiles/r04/experiments/gpu_pcie.txt)."""
    return max(max(up, down) / 57e9, (up + down) / 74.5e9) * 1e3


def host_leg(args, d: Dist, ctx, b: Batch):
    """C2 through wc_forward_host: the cells start in pinned host memory, the
    packed payloads end in pageable host memory; includes both PCIe copies.
    `ms_per_step`: a streaming caller that reuses its output buffers across
    batches; `fresh_ms_per_step`: new output arrays every call, as
    Context.forward_host allocates them (page faults in the call, the previous
    result's free in the loop: the host's mmap/munmap cost, not the link's)."""
    import numpy as np
    import torch
    pinned = torch.empty(b.cells_dev.numel(), dtype=b.cells_dev.dtype, pin_memory=True)
    pinned.copy_(b.cells_dev)
    torch.cuda.synchronize()
    arr = pinned.numpy()
    steps = max(1, min(args.leg_steps, 5))
    bufs = (np.empty(b.capi.payload_bound(b.tab, b.n), np.uint8), np.zeros(b.n + 1, np.uint64),
            np.zeros(max(b.n, 1), np.uint32))
    out = np.zeros(arr.size, np.float32)

    def timed(fn):
        fn()  # warm-up: host staging buffers, destination pages
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        return (time.perf_counter() - t0) / steps * 1e3

    ms = timed(lambda: ctx.forward_host(arr, b.tab, b.n, b.keep, out=bufs))
    payload, offs = bufs[0], bufs[1]
    h2d = arr.nbytes
    d2h = int(offs[b.n])
    ims = timed(lambda: ctx.inverse_host(payload, offs[:b.n], b.tab, b.n, arr.size, out=out))
    # fresh result arrays per call (the previous call's freed inside the loop)
    res = {}
    fms = timed(lambda: res.update(r=ctx.forward_host(arr, b.tab, b.n, b.keep)))
    fims = timed(lambda: res.update(o=ctx.inverse_host(payload, offs[:b.n], b.tab, b.n, arr.size)))
    assert np.array_equal(res["r"][0][:d2h + 4], payload[:d2h + 4]) and np.array_equal(res["o"], out[:arr.size])
    # the same four with huge pages advised on the destinations (WC_OPT_HOST_THP 1,
    # opt-in since round 5: it changes the caller's memory policy)
    ctx.set_option(b.capi.WC_OPT_HOST_THP, 1)
    try:
        thp = {"ms_per_step": timed(lambda: ctx.forward_host(arr, b.tab, b.n, b.keep, out=bufs)),
               "fresh_ms_per_step": timed(lambda: res.update(r=ctx.forward_host(arr, b.tab, b.n, b.keep))),
               "inverse_ms_per_step": timed(lambda: ctx.inverse_host(payload, offs[:b.n], b.tab, b.n, arr.size,
                                                                     out=out)),
               "inverse_fresh_ms_per_step": timed(lambda: res.update(
                   o=ctx.inverse_host(payload, offs[:b.n], b.tab, b.n, arr.size)))}
    finally:
        ctx.set_option(b.capi.WC_OPT_HOST_THP, 0)
    del res
    return {"value": b.ncells / (ms * 1e-3), "unit": "cells/s", "ms_per_step": ms,
            "h2d_bytes": h2d, "d2h_bytes": d2h, "host_GBps": (h2d + d2h) / (ms * 1e-3) / 1e9,
            "fresh_ms_per_step": fms,
            "inverse": {"value": b.ncells / (ims * 1e-3), "unit": "cells/s", "ms_per_step": ims,
                        "h2d_bytes": d2h, "d2h_bytes": 4 * b.ncells,
                        "host_GBps": (d2h + 4 * b.ncells) / (ims * 1e-3) / 1e9, "fresh_ms_per_step": fims},
            "link_bound_ms": {"forward": link_ms(h2d, d2h), "inverse": link_ms(d2h, 4 * b.ncells),
                              "note": "max(bytes of the larger direction / 57 GB/s, bytes of both / 74.5 GB/s): "
                                      "the box's measured PCIe rates, one direction and both at once "
                                      "(profiles/r04/experiments/gpu_pcie.txt)"},
            "thp_on": thp,
            "note": "PCIe-inclusive (pinned host cells in, packed payloads out to pageable host buffers), one rank. "
                    "ms_per_step (since round 4): the caller's output buffers REUSED across calls; "
                    "fresh_ms_per_step: new result arrays every call (round 3's ms_per_step definition). "
                    "Compare reused with reused and fresh with fresh. Default WC_OPT_HOST_THP 0; thp_on: 1. "
                    "`value` above is the HBM-resident rate"}


# ---------------------------------------------------------------------------
# CPU baseline (the oracle: checker + reported baseline only)

def host_threads():
    """Threads the CPU baseline uses: this process's CPU share.  On the GPU box
    the job's share is OMP_NUM_THREADS (16 per GPU); nproc shows the whole host."""
    aff = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(aff, omp) if omp > 0 else aff), aff


def cpu_baseline(args, b: Batch, rmse_dev):
    """Oracle restatement (gcc -O2; ctypes releases the GIL) on a bounded sample
    of the same boxes: one thread, then a thread pool over boxes (the
    reference's per-box loop is embarrassingly parallel); then the
    reference-faithful compress() equivalent WITH xz preset 6 / CRC64 (the
    reference's liblzma parameters, src/compressor.cpp:256-291).  The sample's
    payload bytes and per-box RMSE are compared with the GPU's."""
    import lzma
    from concurrent.futures import ThreadPoolExecutor

    import numpy as np
    from oracle import oracle as O

    threads, aff = host_threads()
    off = b.offsets.cpu().numpy()
    kp = b.kept.cpu().numpy()
    host = {}

    def box(i):
        if i not in host:
            u = b.units[i]
            o = b.offs[i]
            host[i] = b.cells_dev[o:o + u.cells].cpu().numpy().reshape(u.D, u.H, u.W)
        return host[i]

    def payload(i):
        x = box(i)
        return O.compress_payload(O.narrow(x) if x.dtype == np.float64 else x, b.keep)[0]

    t_one, done, parity = 0.0, 0, True
    budget = args.cpu_seconds
    while done < b.n and t_one < budget / 2:
        box(done)
        t0 = time.perf_counter()
        want = payload(done)
        t_one += time.perf_counter() - t0
        o = int(off[done])
        parity &= b.payload[o:o + 20 + 8 * int(kp[done])].cpu().numpy().tobytes() == want
        done += 1
    with ThreadPoolExecutor(threads) as ex:
        t_mt, reps = 0.0, 0
        while t_mt < budget / 2:
            t0 = time.perf_counter()
            list(ex.map(payload, range(done)))
            t_mt += time.perf_counter() - t0
            reps += 1
        # compress() with xz preset 6 (~97 % of the reference's time)
        xz_done, t_xz = 0, 0.0
        t0 = time.perf_counter()
        while t_xz < budget and xz_done < done:
            chunk = list(range(xz_done, min(done, xz_done + threads)))
            list(ex.map(lambda i: lzma.compress(payload(i), format=lzma.FORMAT_XZ, check=lzma.CHECK_CRC64,
                                                preset=6), chunk))
            xz_done += len(chunk)
            t_xz = time.perf_counter() - t0
    cells = b.units[0].cells
    # RMSE check: the oracle's decompress + calc_rmse_per_box on a few sampled boxes
    nchk = min(done, 8)
    rmse_ok, rel = True, 0.0
    if rmse_dev is not None:
        rg = rmse_dev[:b.n].cpu().numpy()
        for i in range(nchk):
            o = int(off[i])
            x = box(i)
            want_regen = O.decompress_payload(b.payload[o:o + 20 + 8 * int(kp[i])].cpu().numpy().tobytes())
            want = O.rmse(O.narrow(x) if x.dtype == np.float64 else x, want_regen)
            r = abs(rg[i] - want) / max(abs(want), 1e-300)
            rel = max(rel, r)
            rmse_ok &= r <= 1e-6
    return {"value": reps * done * cells / t_mt, "unit": "cells/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "affinity_cpus": aff,
            "sample": f"first {done} of {b.n} boxes ({done * cells} cells) x {reps} passes over {threads} "
                      f"threads, oracle narrow+transform+threshold+RLE+serialize (no xz), {t_mt:.1f} s",
            "single_thread": {"value": done * cells / t_one, "cores": 1, "seconds": round(t_one, 2)},
            "with_xz": {"value": xz_done * cells / t_xz if t_xz else None, "unit": "cells/s", "cores": threads,
                        "sample": f"{xz_done} boxes, compress() equivalent incl. xz preset 6 / CRC64 "
                                  f"(python lzma = liblzma), {t_xz:.1f} s"},
            "sample_parity": bool(parity),
            "rmse_check": {"boxes": nchk, "max_rel_diff": rel, "within_1e-6": bool(rmse_ok)}}


# ---------------------------------------------------------------------------
# opt-in legs: the command line and the literal drop-in path, in their own processes

def _cpu_compress_rate(cpu):
    """The reference's compress() work (transform ... serialize + xz preset 6)
    per host thread, from cpu_baseline.with_xz (xz is per unit, so the pool's
    rate / its threads is the single-thread rate)."""
    try:
        wx = cpu["with_xz"]
        return wx["value"] / max(1, wx["cores"])
    except (TypeError, KeyError):
        return None


def _last_json(text):
    for ln in reversed(text.splitlines()):
        if ln.startswith("{"):
            return json.loads(ln)
    raise RuntimeError("no JSON line in:\n" + text[-2000:])


def cli_leg(args, cpu):
    """End-to-end -c / -d / -estimate of the CLI on a C3-like plotfile (tools/bench_cli.py)."""
    out = ROOT / "gpurun_out" / "cli_e2e.json"
    cmd = [sys.executable, str(ROOT / "tools" / "bench_cli.py"), "--scale", "1.0", "--ncomp", "4", "--out", str(out)]
    rate = _cpu_compress_rate(cpu)
    if rate:
        cmd += ["--cpu-cells-per-s", str(rate)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1500)
    if r.returncode:
        return {"error": r.stderr[-2000:]}
    res = _last_json(r.stdout)
    res.pop("cli_logs", None)
    return res


def dropin_leg(args, cpu):
    """INTEGRATION.md Option A: the reference's per-box loops over the C++ mirror
    (compress() per box, decompress() per file) on the C3 layout, 4 fp32
    components per box (tools/dropin_bench.cpp), beside the CPU rate of the
    reference's compress() work per box (single thread, xz preset 6)."""
    import tempfile
    exe = ROOT / "tools" / "bin" / "dropin_bench"
    with tempfile.TemporaryDirectory(prefix="wcamd_dropin_") as d:
        r = subprocess.run([str(exe), d + "/files", "4", "0.999"], capture_output=True, text=True, timeout=1500)
    if r.returncode:
        return {"error": r.stderr[-2000:]}
    res = _last_json(r.stdout)
    rate = _cpu_compress_rate(cpu)
    if rate:
        res["cpu_compress_single_thread"] = {
            "cells_per_s": rate, "ms_per_box": res["cells"] / res["boxes"] / rate * 1e3,
            "note": "the reference's compress() work per host thread (cpu_baseline.with_xz / its threads: oracle "
                    "transform+threshold+RLE+serialize + xz preset 6), per box of this layout's mean size"}
        res["speedup_vs_cpu_single_thread"] = res["compress_cells_per_s"] / rate
        if isinstance(res.get("write_behind"), dict):
            res["write_behind"]["speedup_vs_cpu_single_thread"] = res["write_behind"]["compress_cells_per_s"] / rate
    return res


def plumbing_run(args, d: Dist):
    """CPU check of the launcher: ranks, shard plans and the metric reduction."""
    import bench_workloads as bw
    shards = {}
    for name in ("c5", "c4"):
        units, span = rank_units(name, d)
        m = d.reduce({"cells": sum(u.cells for u in units), "boxes": len(units),
                      "max_rank_cells": sum(u.cells for u in units)})
        shards[name] = {"rank0_span": list(span), "units_total": int(m["boxes"]),
                        "cells_total": int(m["cells"]),
                        "expected_total": sum(u.cells for u in bw.WORKLOADS[name]["units"]())}
    m = d.reduce({"seconds": 0.001 * (d.rank + 1), "boxes": 1})
    return {"metric": "plumbing (no kernels)", "value": None, "n_gpus": d.world, "ranks_seen": int(m["boxes"]),
            "max_seconds": m["seconds"], "shards": shards, "dist_backend": d.backend()}


def main():
    args = parse()
    import wcamd  # noqa: F401  (registers the package as wavelet_compression_amd; no GPU call)
    args.legs_set = set() if args.legs in ("none", "") else set(args.legs.split(","))
    if (args.gpus > 1 or args.force_dist) and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))
    d = Dist(args.plumbing, args.rehearse, args.dist_timeout, args.force_dist)
    if args.plumbing:
        if d.rank == args.fail_rank:
            raise RuntimeError(f"rank {d.rank}: injected failure before the first collective (--fail-rank)")
        out = plumbing_run(args, d)
        if d.rank == 0:
            print(json.dumps(out), flush=True)
        d.close()
        return
    import torch
    import wcamd
    ctx = new_context(args, d)
    out, b = headline(args, d, ctx)
    if "inverse" in args.legs_set:
        out["inverse"] = inverse_leg(args, d, ctx, b)
    if "host" in args.legs_set and d.world == 1:
        out["host"] = host_leg(args, d, ctx, b)
    out["cpu_baseline"] = None
    if d.rank == 0 and d.world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, b, b.rmse)
    ctx.close()
    del b
    torch.cuda.empty_cache()
    if "c3" in args.legs_set and d.world == 1:
        out["c3"] = round_trip_leg(args, d, "c3")
    if "f32_64" in args.legs_set:
        out["f32_64"] = sharded_forward_leg(args, d, "f32_64")
    if "c5" in args.legs_set:
        out["c5"] = sharded_forward_leg(args, d, "c5", inverse=True)
    if "c4" in args.legs_set:
        out["c4"] = sharded_forward_leg(args, d, "c4", hist=True)
    if d.world == 1 and "cli" in args.legs_set:
        out["cli"] = cli_leg(args, out.get("cpu_baseline"))
    if d.world == 1 and "dropin" in args.legs_set:
        out["dropin"] = dropin_leg(args, out.get("cpu_baseline"))
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()
