"""Per-kernel SQ cycle breakdown from a rocprofv3 --pmc counter_collection.csv
(tools/gpu_sq.sh): averages over the dispatches of each kernel, and the shares
of SQ_WAVE_CYCLES spent parked (SQ_WAIT_ANY: s_waitcnt / barrier), issue-stalled
(SQ_WAIT_INST_ANY) and issuing (SQ_ACTIVE_INST_ANY), MI355X_MICROARCH.md §PMC.

usage: python tools/sq_summary.py gpurun_out/sq3/c2_counter_collection.csv [...]
"""
import collections
import csv
import re
import sys

SHORT = [("k_transform_fast", "K1 transform"), ("k_transform_fallback", "K1b fallback"), ("k_emit", "K2 emit"),
         ("k_rowindex", "K5 row index"), ("k_pair_counts", "K5p header check"), ("k_inverse_rows", "K6r inverse"),
         ("k_rmse", "K7 rmse")]


def short(name: str) -> str:
    for key, label in SHORT:
        if key in name:
            m = re.search(key + r"<([^>]*)>", name)
            return f"{label}<{m.group(1)}>" if m else label
    return ""


def main(paths):
    for path in paths:
        per = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            if k:
                per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        print(f"== {path}")
        for k, cs in per.items():
            avg = {c: sum(v) / len(v) for c, v in cs.items()}
            wc = avg.get("SQ_WAVE_CYCLES", 0.0)
            line = f"  {k:28s} waves {avg.get('SQ_WAVES', 0):9.0f}  wave-cycles {wc:12.4g}"
            if wc:
                for c, lab in (("SQ_WAIT_ANY", "parked"), ("SQ_WAIT_INST_ANY", "issue-stall"),
                               ("SQ_ACTIVE_INST_ANY", "issuing"), ("SQ_WAIT_INST_LDS", "lds-stall")):
                    if c in avg:
                        line += f"  {lab} {avg[c] / wc:5.1%}"
            if avg.get("SQ_LDS_IDX_ACTIVE"):
                line += f"  lds-conflict/lds-active {avg.get('SQ_LDS_BANK_CONFLICT', 0) / avg['SQ_LDS_IDX_ACTIVE']:5.1%}"
            print(line)


if __name__ == "__main__":
    main(sys.argv[1:])
