"""Multi-GPU sharding of independent units.

A unit (time, level, box, component) is fully independent in the reference:
its threshold is box-local (src/compressor.cpp:212-216) and it gets its own
output file (:250-254).  So the batch is split into contiguous unit ranges,
one per rank (one process per GPU), balanced by cell count, with no
data-path collective.  The only collective is one small all-reduce of the run
metrics (kept counts, payload bytes, per-component min/max and RMSE sums),
which over RCCL is a few hundred bytes and latency-bound.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple


def plan_shards(cell_counts: Sequence[int], world: int) -> List[Tuple[int, int]]:
    """Split units [0, n) into `world` contiguous ranges with near-equal cells.

    Boundary r is the first unit whose cell prefix reaches r/world of the total,
    so ranges stay in unit order (rank r's payloads precede rank r+1's) and the
    largest range exceeds the ideal share by at most one unit."""
    n = len(cell_counts)
    if world < 1:
        raise ValueError("world must be >= 1")
    total = sum(int(c) for c in cell_counts)
    bounds = [0]
    prefix = 0
    i = 0
    for r in range(1, world):
        target = total * r / world
        while i < n and prefix + int(cell_counts[i]) / 2 < target:
            prefix += int(cell_counts[i])
            i += 1
        bounds.append(max(i, bounds[-1]))
    bounds.append(n)
    return [(bounds[r], bounds[r + 1]) for r in range(world)]


METRIC_SUM = ("cells", "kept", "payload_bytes", "rmse_sum", "boxes")


def reduce_metrics(local: Dict[str, float], group=None, device=None) -> Dict[str, float]:
    """All-reduce run metrics across ranks: sums for METRIC_SUM keys, MAX for
    'seconds' and 'max_*', MIN for 'min_*'.  One tensor per reduction op."""
    import torch
    import torch.distributed as dist

    keys = sorted(local)
    sums = [k for k in keys if k in METRIC_SUM]
    maxs = [k for k in keys if k == "seconds" or k.startswith("max_")]
    mins = [k for k in keys if k.startswith("min_")]
    out = dict(local)
    for ks, op in ((sums, dist.ReduceOp.SUM), (maxs, dist.ReduceOp.MAX), (mins, dist.ReduceOp.MIN)):
        if not ks:
            continue
        t = torch.tensor([float(local[k]) for k in ks], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=op, group=group)
        out.update({k: float(v) for k, v in zip(ks, t.tolist())})
    return out


def global_threshold(ctx, d_cells: int, dtype: int, units, n: int, quantile: float, hist, group=None):
    """Opt-in global-threshold mode (include/wavelet_amd.h wc_forward_stage):
    transform this rank's units, add their coefficient-magnitude histogram to
    `hist` (a zeroed int64 torch tensor of capi.HIST_BINS bins on this rank's
    device, reinterpreted as uint64 by the library), sum it over ranks with ONE
    all-reduce (RCCL over xGMI on GPUs, gloo on CPU) and return
    (fp32 threshold, retained count over all ranks).  Follow with
    ctx.forward_emit(units, n, keep, threshold, ...).

    Not the reference's rule (a per-box max threshold, src/compressor.cpp:212-216):
    the retained index set differs from the reference by design."""
    import numpy as np
    import torch.distributed as dist

    from . import capi

    ctx.forward_stage(d_cells, dtype, units, n, hist.data_ptr())
    ctx.synchronize()  # the context stream may not be the collective's stream
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    h = hist.cpu().numpy().view(np.uint64)
    return capi.hist_threshold(h, quantile)
