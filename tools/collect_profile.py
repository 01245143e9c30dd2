"""Copy one `tools/gpu_profile.sh` call's outputs from gpurun_out/ into profiles/<round>/.

usage: python tools/collect_profile.py <log> [--round r05]

* pmc_<w>.json and the wc_bench kernel traces of every workload, the bench.py trace, the bench
  line, cli_e2e.json;
* dropin.json with the single-thread CPU compress() rate of the same call merged in (bench.py's
  cpu_baseline.with_xz divided by its threads, per box of the layout's mean size);
* gpu_tests.txt: the `-m gpu` suite's output from the call's log (GPUTEST=1), headed by the
  kernel-source hash and the commit the pmc summaries recorded.
"""
import argparse
import json
import shutil
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
OUT = ROOT / "gpurun_out"
WORKLOADS = ("c2", "c3", "c4", "c5", "f32_64", "c4_hist")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("log")
    ap.add_argument("--round", default="r06")
    a = ap.parse_args()
    dst = ROOT / "profiles" / a.round
    dst.mkdir(parents=True, exist_ok=True)
    for w in WORKLOADS:
        shutil.copy(OUT / "pmc" / f"pmc_{w}.json", dst / f"pmc_{w}.json")
        shutil.copy(OUT / f"prof_{w}" / "kt_kernel_stats.csv", dst / f"kernel_stats_wc_bench_{w}.csv")
    shutil.copy(OUT / "prof_bench" / "bench_kernel_stats.csv", dst / "kernel_stats_bench_py.csv")
    shutil.copy(OUT / "bench_line.txt", dst / "bench_line.txt")
    if (OUT / "cli_e2e.json").exists():
        shutil.copy(OUT / "cli_e2e.json", dst / "cli_e2e.json")
    line = json.loads((OUT / "bench_line.txt").read_text().strip().splitlines()[-1])
    pmc = json.loads((dst / "pmc_c2.json").read_text())
    if (OUT / "dropin.json").exists():
        d = json.loads((OUT / "dropin.json").read_text())
        wx = line["cpu_baseline"]["with_xz"]
        per = wx["value"] / wx["cores"]
        d["command"] = ("tools/bin/dropin_bench <scratch> 4 0.999 (tools/gpu_profile.sh DROPIN=1, same call as "
                        "bench_line.txt)")
        d["cpu_compress_single_thread"] = {
            "cells_per_s": per, "ms_per_box": d["cells"] / d["boxes"] / per * 1e3,
            "note": ("the reference's compress() work per host thread (bench.py cpu_baseline.with_xz / its threads, "
                     "same call: oracle transform+threshold+RLE+serialize + xz preset 6), per box of this layout's "
                     "mean size")}
        d["speedup_vs_cpu_single_thread"] = d["compress_cells_per_s"] / per
        if "write_behind" in d:
            d["write_behind"]["speedup_vs_cpu_single_thread"] = d["write_behind"]["compress_cells_per_s"] / per
        (dst / "dropin.json").write_text(json.dumps(d, indent=1))
    log = Path(a.log).read_text().splitlines()
    rc = [i for i, s in enumerate(log) if s.startswith("== gputest rc=")]
    if rc:
        full = OUT / "gputest.log"  # the suite's whole output (the call's log holds its tail)
        body = (full.read_text().splitlines() if full.exists()
                else [s for s in log[rc[0] + 1:] if not s.startswith("== ")])
        head = (f"# python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread (tools/gpu_profile.sh "
                f"GPUTEST=1, kernel-source hash {pmc['kernel_sources_sha']}, commit {pmc['git']})")
        (dst / "gpu_tests.txt").write_text("\n".join([head] + body) + "\n")
    bad = [s for s in log if s.startswith("== ") and " rc=" in s and " rc=0 " not in s]
    print(f"collected into {dst} (hash {pmc['kernel_sources_sha']}, commit {pmc['git']})"
          + (f"; steps that failed: {bad}" if bad else ""))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
