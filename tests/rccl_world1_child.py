"""Child of tests/test_gpu_rccl.py, started by torch.distributed.run
(--nproc-per-node 1) BEFORE anything in it touches the GPU: the RCCL backend
at world 1 on the one-GPU box, each collective the multi-GPU path uses
(bench.py Dist, shard.py) checked against the no-dist path:

  * init_process_group("nccl", device_id=...)        (bench.py Dist)
  * reduce_metrics: float64 SUM / MAX / MIN on a CUDA tensor (shard.py)
  * global_threshold: the int64 4096-bin histogram all-reduce on the C4 batch
    (the opt-in global-threshold mode), against forward_stage with no collective
  * all_gather_object over the NCCL group (bench.py Dist.gather)
  * barrier

Prints ONE JSON line with the results; the parent asserts on it.
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    import datetime

    import numpy as np
    import torch
    import torch.distributed as dist

    local = int(os.environ["LOCAL_RANK"])
    dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=datetime.timedelta(seconds=120))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    out = {"backend": dist.get_backend(), "world": dist.get_world_size(), "rank": dist.get_rank()}

    import wcamd
    import bench_workloads as bw
    from wavelet_compression_amd.shard import global_threshold, reduce_metrics

    # float64 SUM / MAX / MIN over RCCL on a CUDA tensor
    local_m = {"cells": 3.0e9, "kept": 123456789.0, "boxes": 46080.0, "rmse_sum": 0.125,
               "seconds": 0.0133, "max_rank_cells": 7.5e8, "min_rank_cells": 6.25e8}
    red = reduce_metrics(local_m, device=dev)
    out["reduce_equal"] = red == local_m

    # the C4 batch's magnitude histogram: no collective, then through global_threshold
    units = bw.WORKLOADS["c4"]["units"]()
    cells, offs, _ = bw.synth_cells(torch, dev, units, "f64")
    tab, n, _ = bw.units_array(wcamd.capi, units, offs)
    ctx = wcamd.capi.Context(local)
    h0 = torch.zeros(wcamd.capi.HIST_BINS, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    ctx.forward_stage(cells.data_ptr(), wcamd.capi.WC_F64, tab, n, h0.data_ptr())
    ctx.synchronize()
    want = h0.cpu().numpy().view(np.uint64).copy()
    t0, r0 = wcamd.capi.hist_threshold(want, 0.7)
    h1 = torch.zeros_like(h0)
    torch.cuda.synchronize()
    t1, r1 = global_threshold(ctx, cells.data_ptr(), wcamd.capi.WC_F64, tab, n, 0.7, h1)
    got = h1.cpu().numpy().view(np.uint64)
    total = sum(u.cells for u in units)
    out.update(units=n, cells=total, hist_equal=bool(np.array_equal(got, want)),
               hist_total=int(want.sum()), threshold=[t0, t1], retained=[r0, r1])
    ctx.close()

    # all_gather_object over the NCCL group, then a barrier
    g = [None]
    dist.all_gather_object(g, {"rank": dist.get_rank(), "retained": r1})
    out["gather"] = g
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
