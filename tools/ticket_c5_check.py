"""Diagnostic: C5 (512 x 128^3 fp32, keep 0.9999f) through wc_forward in the
look-backs' ticket form, against the launch-order form's kept counts.
Round-4 GPU suite: test_gpu_c5.py::test_c5_paths_identical_all_units[2-2]
(a second context alive -> ticket form) returned kept == 0 for tail units
with no error.  This runs the same batch several ways in one process and
prints, per call, how many units differ and where."""
import json
import sys

import numpy as np

sys.path.insert(0, ".")
import torch  # noqa: E402

import bench_workloads as bw  # noqa: E402
import wcamd  # noqa: E402
from wavelet_compression_amd.capi import WC_OPT_COHORT, WC_OPT_ORDERED  # noqa: E402

wc = wcamd
KEEP = float(np.float32(0.9999))
dev = torch.device("cuda", 0)
units = bw.WORKLOADS["c5"]["units"]()
cells, offs, extent = bw.synth_cells(torch, dev, units, "f32")
tab, n, _ = bw.units_array(wc.capi, units, offs)
cap = wc.capi.payload_bound(tab, n)
payload = torch.zeros(cap, dtype=torch.uint8, device=dev)
offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
kept = torch.zeros(n, dtype=torch.int32, device=dev)


def run(c, label):
    payload.zero_()
    offsets.zero_()
    kept.zero_()
    torch.cuda.synchronize()
    err = None
    try:
        c.forward(cells.data_ptr(), wc.capi.WC_F32, tab, n, KEEP, payload.data_ptr(), cap, offsets.data_ptr(),
                  kept.data_ptr())
        c.synchronize()
    except wc.WaveletError as e:
        err = str(e)
    k = kept.cpu().numpy().copy()
    return label, k, err, offsets.cpu().numpy().copy()


a = wc.capi.Context(0)
ref = run(a, "ordered, one context")
print(json.dumps({"call": ref[0], "err": ref[2], "zeros": int((ref[1] == 0).sum()), "kept_sum": int(ref[1].sum())}),
      flush=True)
results = []
a.set_option(WC_OPT_ORDERED, 0)
for i in range(3):
    results.append(run(a, f"tickets (WC_OPT_ORDERED 0), one context #{i}"))
a.set_option(WC_OPT_ORDERED, 1)
b = wc.capi.Context(0)  # two live contexts: both take the ticket form
for i in range(3):
    results.append(run(b, f"second context, cohort 0 #{i}"))
b.set_option(WC_OPT_COHORT, 2)
for i in range(3):
    results.append(run(b, f"second context, cohort 2 (ticket form) #{i}"))
for label, k, err, o in results:
    bad = np.nonzero(k != ref[1])[0]
    print(json.dumps({"call": label, "err": err, "units_differ": int(bad.size),
                      "first": bad[:8].tolist(), "zeros": int((k == 0).sum()),
                      "offsets_differ": int((o != ref[3]).sum())}), flush=True)
b.close()
a.close()
