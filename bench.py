"""bench.py — forward hot path (transform + keep threshold + ordered pack) on MI355X.

Workload (BASELINE.json configs[1]): 1024 synthetic 64^3 fp64 boxes per GPU,
1 component, keep = 0.999f, inputs resident in HBM before the timed region.
One step = one wc_forward over the whole batch (cells -> serialized payloads).
Multi-GPU: one process per GPU; every rank compresses its own 1024 boxes
(independent AMR units, no data-path collective) -> weak scaling.  The only
collective is a small all-reduce of kept/byte counts after timing.

Prints ONE JSON line on rank 0 (driver contract).  The CPU baseline is the
oracle restatement (single thread) on a bounded sample of the same boxes; the
sample's payload bytes are also compared with the GPU's ("sample_parity").
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

PEAK_HBM_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--boxes", type=int, default=1024)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--dtype", choices=("f64", "f32"), default="f64")
    ap.add_argument("--keep", type=float, default=0.999)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="time budget of the CPU-baseline sample (boxes run until it is spent)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pmc", default=str(ROOT / "profiles" / "r01" / "pmc_forward.json"),
                    help="PMC traffic summary (tools/pmc_summary.py) merged into roofline.traffic")
    ap.add_argument("--pipe", action="store_true", help="run the pipelined single-launch forward (WC_OPT_PIPE)")
    ap.add_argument("--no-inverse", action="store_true", help="skip the inverse-path figures")
    ap.add_argument("--hist-quantile", type=float, default=None,
                    help="also time the opt-in global-threshold mode (NOT the reference rule): stage + "
                         "magnitude histogram, one all-reduce over ranks (RCCL), threshold at this quantile, emit")
    return ap.parse_args()


def synth_device(torch, dev, nboxes, dim, dtype, rank):
    """v = 300 + 50 sin(0.1 gx) cos(0.07 gy) + 0.01 gz + 0.05 N(0,1)  (SURVEY.md §8(d)),
    boxes tiled over a 16 x 8 x (n/128) grid of 64^3 patches, generated on device."""
    td = torch.float64 if dtype == "f64" else torch.float32
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + 7919 * rank)
    n = dim
    z = torch.arange(n, device=dev, dtype=torch.float64).view(n, 1, 1)
    y = torch.arange(n, device=dev, dtype=torch.float64).view(1, n, 1)
    x = torch.arange(n, device=dev, dtype=torch.float64).view(1, 1, n)
    out = torch.empty(nboxes * n ** 3, dtype=td, device=dev)
    for b in range(nboxes):
        lx, ly, lz = n * (b % 16), n * ((b // 16) % 8), n * (b // 128) + 4096 * rank
        v = 300.0 + 50.0 * torch.sin(0.1 * (x + lx)) * torch.cos(0.07 * (y + ly)) + 0.01 * (z + lz)
        v = v + 0.05 * torch.randn((n, n, n), generator=g, device=dev, dtype=torch.float64)
        out[b * n ** 3:(b + 1) * n ** 3] = v.reshape(-1).to(td)
    return out


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    import wcamd
    capi = wcamd.capi
    ctx = capi.Context(local)
    ctx.set_pipe(args.pipe)
    keep = float(np.float32(args.keep))  # Config::keep is a float (src/argparse.h:13)
    dims = [(args.dim,) * 3] * args.boxes
    units, n, extent = capi.make_units(dims)
    ncells = extent  # dense, 64^3 multiples: no padding
    dtype_code = capi.WC_F64 if args.dtype == "f64" else capi.WC_F32
    s_in = 8 if args.dtype == "f64" else 4

    cells = synth_device(torch, dev, args.boxes, args.dim, args.dtype, rank)
    cap = capi.payload_bound(units, n)
    payload = torch.empty(cap, dtype=torch.uint8, device=dev)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    kept = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def step():
        ctx.forward(cells.data_ptr(), dtype_code, units, n, keep, payload.data_ptr(), cap,
                    offsets.data_ptr(), kept.data_ptr())

    for _ in range(args.warmup):
        step()
    ctx.synchronize()

    # Timed region: no per-kernel events (they would sit between the launches).
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()

    # Per-kernel launch times (hipEvents on the context's stream, where the
    # kernels run) from the same number of steps right after.
    ctx.profile_enable(True)
    ctx.profile_read()  # reset
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    ctx.profile_enable(False)
    stages = ctx.profile_read()

    elapsed = t1 - t0
    kept_total = int(kept.sum().item())
    payload_bytes = int(kept.to(torch.int64).sum().item()) * 8 + 20 * n  # serialized bytes (slots excluded)
    local = {"seconds": elapsed, "kept": kept_total, "payload_bytes": payload_bytes, "cells": ncells}
    if world > 1:
        # the one collective: run metrics (a few bytes) over RCCL, after timing
        from wavelet_compression_amd.shard import reduce_metrics
        local = reduce_metrics(local, device=dev)
    elapsed = local["seconds"]
    kept_all, bytes_all, cells_all = local["kept"], local["payload_bytes"], local["cells"]

    # ---- roofline of the dominant kernel (per-launch averages from hipEvents) ----
    per_launch = {k: (ms / cnt, cnt) for k, (ms, cnt) in stages.items()}
    dominant = max(per_launch, key=lambda k: per_launch[k][0])
    kept_step = kept_total  # per launch (this rank)
    alg_bytes_stage = {
        # algorithmic bytes each kernel owns of B = s_in*N + 8*N_kept + 20*N_units;
        # the fp32 coefficient staging between K1 and K2 is overhead, not algorithmic traffic.
        "transform": s_in * ncells,
        "flat_emit": 8 * kept_step + 20 * n,
        # the pipelined kernel owns the whole path: cells in, pairs + headers out
        "pipe": s_in * ncells + 8 * kept_step + 20 * n,
    }
    dom_ms = per_launch[dominant][0]
    achieved = alg_bytes_stage.get(dominant, 0) / (dom_ms * 1e-3) / 1e9
    path_ms = sum(v[0] for v in per_launch.values())
    path_bytes = s_in * ncells + 8 * kept_step + 20 * n
    # Reference point for "achievable": a device-to-device copy of the cell
    # buffer (torch's copy kernel, read + write bytes per second).
    scratch = torch.empty_like(cells)
    scratch.copy_(cells)
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(5):
        scratch.copy_(cells)
    ev1.record()
    torch.cuda.synchronize()
    copy_gbps = 2 * cells.numel() * cells.element_size() * 5 / (ev0.elapsed_time(ev1) * 1e-3) / 1e9
    del scratch
    traffic = None
    pmc_path = Path(args.pmc)
    if pmc_path.exists():
        try:
            pmc = json.loads(pmc_path.read_text())
            if pmc.get("config", {}).get("boxes") == args.boxes and pmc.get("config", {}).get("dtype") == args.dtype:
                traffic = pmc.get("per_launch_bytes", {}).get(dominant)
        except Exception:
            traffic = None

    out = {
        "metric": f"{'fp64' if args.dtype == 'f64' else 'fp32'} cells/s, fwd transform+threshold+pack, keep={args.keep}",
        "value": cells_all * args.steps / elapsed,
        "unit": "cells/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (SURVEY §8(d) field + N(0,0.05) noise, generated on device)",
        "config": {"workload": f"{args.boxes}x{args.dim}^3 {args.dtype} boxes/GPU, 1 component, "
                               f"keep={args.keep}f, wc_forward (payload bytes identical to reference)",
                   "boxes_per_gpu": args.boxes, "box_dim": args.dim, "global_batch": args.boxes * world,
                   "parallelism": f"box-sharded x{world}"},
        "compressed_GBps": cells_all * s_in * args.steps / elapsed / 1e9,
        "kept_fraction": kept_all / cells_all,
        "payload_bytes_per_step": bytes_all,
        "stage_ms_per_launch": {k: round(v[0], 4) for k, v in per_launch.items()},
        "roofline": {
            "bound": "hbm", "kernel": dominant,
            "achieved": achieved, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBPS,
            "traffic": traffic,
            # HBM bytes the kernel actually moved (PMC, incl. the fp32 coefficient staging) per second
            "traffic_GBps": (traffic / (dom_ms * 1e-3) / 1e9) if traffic else None,
            "copy_GBps": copy_gbps,
        },
        "roofline_path": {"achieved": path_bytes / (path_ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS,
                          "unit": "GB/s", "frac": path_bytes / (path_ms * 1e-3) / 1e9 / PEAK_HBM_GBPS,
                          "bytes_per_step": path_bytes, "kernel_ms_per_step": path_ms},
        "cpu_baseline": None,
    }

    if not args.no_inverse:
        out["inverse"] = inverse_figures(args, ctx, capi, units, n, ncells, payload, offsets, kept_total, dev)

    if args.hist_quantile is not None:
        out["global_hist"] = global_hist_figures(args, ctx, capi, units, n, dtype_code, cells, payload, cap,
                                                 offsets, kept, dev, world, s_in)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(args, cells, payload, offsets, kept, s_in, keep)

    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def global_hist_figures(args, ctx, capi, units, n, dtype_code, cells, payload, cap, offsets, kept, dev, world,
                        s_in):
    """Opt-in global-threshold mode, timed like the headline step: per step one
    stage (K1 + histogram), ONE all-reduce of the 4096-bin histogram over all
    ranks (RCCL over xGMI when world > 1), the threshold on the host, one emit."""
    import torch
    import torch.distributed as dist
    from wavelet_compression_amd.shard import global_threshold

    hist = torch.zeros(capi.HIST_BINS, dtype=torch.int64, device=dev)
    res = {}

    def step():
        hist.zero_()
        t, r = global_threshold(ctx, cells.data_ptr(), dtype_code, units, n, args.hist_quantile, hist)
        ctx.forward_emit(units, n, 0.0, t, payload.data_ptr(), cap, offsets.data_ptr(), kept.data_ptr())
        res.update(thresh=t, retained=r)

    for _ in range(max(1, args.warmup)):
        step()
    ctx.synchronize()
    ctx.profile_enable(True)
    ctx.profile_read()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    ctx.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    ctx.profile_enable(False)
    stages = ctx.profile_read()
    kept_rank = int(kept.sum().item())
    cells_rank = args.boxes * args.dim ** 3
    m = {"seconds": elapsed, "kept": kept_rank, "cells": cells_rank}
    if world > 1:
        from wavelet_compression_amd.shard import reduce_metrics
        m = reduce_metrics(m, device=dev)
    return {
        "mode": "global histogram threshold (opt-in, not the reference rule)",
        "quantile": args.hist_quantile, "threshold": res["thresh"],
        "retained": res["retained"], "kept_check": m["kept"] == res["retained"],
        "kept_fraction": m["kept"] / m["cells"],
        "value": m["cells"] * args.steps / m["seconds"], "unit": "cells/s",
        "ms_per_step": m["seconds"] / args.steps * 1e3,
        "stage_ms_per_launch": {k: round(ms / cnt, 4) for k, (ms, cnt) in stages.items()},
        "allreduce": f"{capi.HIST_BINS} x u64 over {world} rank(s)" + (" (RCCL)" if world > 1 else " (none)"),
    }


def inverse_figures(args, ctx, capi, units, n, ncells, payload, offsets, kept_total, dev):
    """The inverse path over this step's payloads (wc_inverse: rle_decode + inverse transform),
    timed like the forward; SURVEY §8(d) inverse bytes = 8*N_kept + 20*N_units + 4*N_cells."""
    import torch
    regen = torch.empty(ncells, dtype=torch.float32, device=dev)

    def istep():
        ctx.inverse(payload.data_ptr(), offsets.data_ptr(), units, n, regen.data_ptr())

    for _ in range(2):
        istep()
    ctx.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        istep()
    ctx.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ctx.profile_enable(True)  # per-kernel times from a separate loop (events off in the timed one)
    ctx.profile_read()
    for _ in range(args.steps):
        istep()
    ctx.synchronize()
    ctx.profile_enable(False)
    st = ctx.profile_read()
    ms = (t1 - t0) / args.steps * 1e3
    alg = 8 * kept_total + 20 * n + 4 * ncells
    per = {k: v[0] / v[1] for k, v in st.items()}
    return {"value": ncells / (ms * 1e-3), "unit": "cells/s", "ms_per_step": ms,
            "stage_ms_per_launch": {k: round(v, 4) for k, v in per.items()},
            "roofline_path": {"achieved": alg / (ms * 1e-3) / 1e9, "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                              "frac": alg / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, "bytes_per_step": alg}}


def cpu_baseline(args, cells, payload, offsets, kept, s_in, keep):
    """Oracle restatement (gcc -O2; ctypes releases the GIL) on a bounded sample of the same
    boxes: one thread, then a thread pool over boxes (the reference's per-box loop is
    embarrassingly parallel).  The sample's payload bytes are compared with the
    GPU's ("sample_parity")."""
    import numpy as np
    from concurrent.futures import ThreadPoolExecutor
    from oracle import oracle as O  # checker / CPU baseline leg only

    nb = args.dim ** 3
    off = offsets.cpu().numpy()
    kp = kept.cpu().numpy()
    threads = max(1, min(16, len(os.sched_getaffinity(0))))

    def one(i):
        box = host[i]
        b32 = O.narrow(box) if box.dtype == np.float64 else box
        return O.compress_payload(b32, keep)[0]

    # single thread: boxes until half the budget is spent
    host, t_one, done, parity = {}, 0.0, 0, True
    while done < args.boxes and t_one < args.cpu_seconds / 2:
        host[done] = cells[done * nb:(done + 1) * nb].cpu().numpy().reshape((args.dim,) * 3)
        t0 = time.perf_counter()
        want = one(done)
        t_one += time.perf_counter() - t0
        o = int(off[done])
        parity &= payload[o:o + 20 + 8 * int(kp[done])].cpu().numpy().tobytes() == want
        done += 1
    # thread pool: the same boxes, repeated until the other half is spent
    with ThreadPoolExecutor(threads) as ex:
        t_mt, reps = 0.0, 0
        while t_mt < args.cpu_seconds / 2:
            t0 = time.perf_counter()
            list(ex.map(one, range(done)))
            t_mt += time.perf_counter() - t0
            reps += 1
    return {"value": reps * done * nb / t_mt, "unit": "cells/s", "cores": threads, "kind": "port",
            "sample": f"first {done} of {args.boxes} boxes ({done * nb} cells) x {reps} passes over {threads} "
                      f"threads, oracle narrow+transform+threshold+RLE+serialize (no xz), {t_mt:.1f} s",
            "single_thread": {"value": done * nb / t_one, "cores": 1, "seconds": round(t_one, 2)},
            "sample_parity": bool(parity)}


if __name__ == "__main__":
    main()
