"""The RCCL backend at world 1 on the one-GPU box: the
driver's 8-GPU run must not be RCCL's first execution.  Both children are
started with torch.distributed.run in a fresh process (never by exec from this
one, which has touched the GPU), so their process group is set up before any
GPU call, as bench.py's ranks are.

  * tests/rccl_world1_child.py: nccl init with device_id, reduce_metrics'
    float64 SUM / MAX / MIN on a CUDA tensor, shard.global_threshold's int64
    4096-bin all-reduce on the C4 batch, all_gather_object, barrier — each
    equal to the no-dist result;
  * bench.py --force-dist: the Dist nccl branch at world 1 through the c4 leg
    (barriers around every timed region, metric reductions, per-rank gather,
    the histogram all-reduce of the global-threshold mode).
"""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _json(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-3000:]
    return json.loads(lines[0])


def test_rccl_world1_collectives_equal_no_dist_path(tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", str(ROOT / "tests" / "rccl_world1_child.py")]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=110, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["backend"] == "nccl" and out["world"] == 1 and out["rank"] == 0
    assert out["reduce_equal"] is True
    assert out["units"] == 46080 and out["hist_equal"] is True
    assert out["hist_total"] == out["cells"]  # every coefficient binned (no NaN in the field)
    assert out["threshold"][0] == out["threshold"][1] and out["retained"][0] == out["retained"][1]
    assert out["gather"] == [{"rank": 0, "retained": out["retained"][1]}]


def test_bench_force_dist_runs_rccl_at_world1(tmp_path):
    cmd = [sys.executable, str(ROOT / "bench.py"), "--force-dist", "--steps", "2", "--warmup", "1",
           "--leg-steps", "1", "--legs", "c4", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=110, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _json(r.stdout)
    assert out["n_gpus"] == 1 and out["dist_backend"] == "RCCL over xGMI"
    assert out["value"] > 0 and 0.25 < out["kept_fraction"] < 0.35
    c4 = out["c4"]
    assert c4["units_total"] == 46080 and [p["units"] for p in c4["per_rank"]] == [46080]
    gh = c4["global_hist"]
    assert gh["kept_check"] is True and "RCCL over xGMI" in gh["allreduce"]
