"""Summarise tools/gpu_ab.sh logs: per variant and shape, ms/step and stage times."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "ab_*.log"))):
    name = os.path.basename(f)[3:-4]
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(name, "unparsed", e)
        continue
    key = name.rsplit("_", 1)[0] if name[-2] == "_" else name
    rows[key].append(d)
for key, ds in rows.items():
    fw = [d["ms_per_step"] for d in ds]
    st = {k: [round(d["stage_ms"][k], 4) for d in ds] for k in ds[0]["stage_ms"]}
    inv = {k: [round(d.get("inverse_stage_ms", {}).get(k, 0), 4) for d in ds] for k in ds[0].get("inverse_stage_ms", {})}
    print(f"{key:22s} fwd {fw} {st} inv {inv} identical={ds[0].get('paths_identical')}")
for f in sorted(glob.glob(os.path.join(root, "pmc_ab", "*_counter_collection.csv"))):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[(r["Kernel_Name"][:26], r["Counter_Name"])].append(float(r["Counter_Value"]))
    print(os.path.basename(f), {f"{k[0]}|{k[1]}": round(sum(v) / len(v)) for k, v in agg.items() if "synth" not in k[0]})
