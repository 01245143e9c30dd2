"""Regenerate tests/golden/codec_golden.{npz,json} from the CPU oracle.

The oracle (oracle/wc_oracle.c) is pinned by tests/test_oracle.py against the
reference's own known answers and a numpy restatement; these fixtures freeze
its outputs so GPU parity tests can also compare against stored vectors.
Cases follow SURVEY.md §8(c): seeded boxes {2^3, 8x4x2, 6x10x14, 3x4x2 (odd),
16^3, 32^3, 16x32x64} x keep {0.99f, 0.999f, 0.9999f}, special boxes
(sign quirk, +M/-M tie, all-zero, NaN-first), and SHA-256 of the payloads of
seeded 64^3 and 128^3 boxes.

usage: python tests/golden/make_golden.py
"""
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))
from oracle import oracle as O  # noqa: E402

KEEPS = [float(np.float32(k)) for k in (0.99, 0.999, 0.9999)]
DIMS = [(2, 2, 2), (8, 4, 2), (6, 10, 14), (3, 4, 2), (16, 16, 16), (32, 32, 32), (16, 32, 64)]


def main():
    arrays, cases = {}, []

    def add(name, box, keep, box_key=None):
        payload, kept = O.compress_payload(box, keep)
        box_key = box_key or name + "/box"
        arrays.setdefault(box_key, box)
        arrays[name + "/payload"] = np.frombuffer(payload, np.uint8)
        arrays[name + "/regen"] = O.decompress_payload(payload)
        cases.append({"name": name, "box": box_key, "dims": list(box.shape[::-1]), "keep": keep,
                      "kept": kept, "payload_bytes": len(payload)})

    for i, (W, H, D) in enumerate(DIMS):
        cells = O.synth_box_f64(O.unit_seed(0, 0, i, 0), (W * i, H * i, D * i), W, H, D)
        box = O.narrow(cells)
        for k in KEEPS:
            add(f"synth_{W}x{H}x{D}_keep{k:.6g}", box, k, box_key=f"synth_{W}x{H}x{D}/box")
    k = KEEPS[1]
    spike = np.full((4, 4, 4), 5.0, np.float32); spike[1, 2, 3] = 7.5
    add("sign_plus5_spike", spike, k)
    add("sign_minus5", np.full((4, 4, 4), -5.0, np.float32), k)
    tie = np.zeros((4, 4, 8), np.float32); tie[0, 0, 0] = 3.0; tie[0, 0, 1] = -3.0
    add("tie_pm3", tie, k)
    add("all_zero", np.zeros((4, 6, 8), np.float32), k)
    nanf = np.full((8, 4, 4), 2.0, np.float32); nanf[:2, :2, :2] = np.nan
    add("nan_first", nanf, k)

    hashes = []
    for (dim, keep, i) in ((64, KEEPS[1], 0), (128, KEEPS[2], 1)):
        seed = O.unit_seed(0, 0, i, 0)
        cells = O.synth_box_f64(seed, (0, 0, 0), dim, dim, dim)
        payload, kept = O.compress_payload(O.narrow(cells), keep)
        hashes.append({"dims": [dim] * 3, "seed": seed, "lo": [0, 0, 0], "keep": keep, "kept": kept,
                       "payload_sha256": hashlib.sha256(payload).hexdigest()})

    np.savez_compressed(HERE / "codec_golden.npz", **arrays)
    (HERE / "codec_golden.json").write_text(json.dumps({"cases": cases, "hashes": hashes}, indent=1) + "\n")
    print(f"{len(cases)} cases, {len(hashes)} hashes")


if __name__ == "__main__":
    main()
