"""Fit the headline kernel's time per launch against batch (a batch sweep of bench.py --batch lines):
t(batch) = t0 + batch / R by least squares over the launch_b<k>.json bench lines.
Usage: python tools/launch_fit.py gpurun_out/r3d [out.json]"""
import glob
import json
import os
import sys

import numpy as np

d = sys.argv[1]
rows = []
for f in sorted(glob.glob(os.path.join(d, "launch_b*.json"))):
    line = json.load(open(f))
    rows.append((line["config"]["batch_per_gpu"], line["roofline"]["avg_kernel_ms"], line["value"],
                 line["parity"]["bit_exact"]))
rows.sort()
b = np.array([r[0] for r in rows], float)
t = np.array([r[1] for r in rows], float)
A = np.stack([np.ones_like(b), b], 1)
(t0, k), *_ = np.linalg.lstsq(A, t, rcond=None)
bytes_per_transform = 1024 * 16
out = {"points": [{"batch": int(r[0]), "ms_per_launch": r[1], "gsamples_per_s": r[2], "bit_exact": r[3]} for r in rows],
       "fit": {"t0_us": t0 * 1e3, "steady_tb_per_s": bytes_per_transform / (k * 1e-3) * 1e-12,
               "note": "t = t0 + batch * 16 KiB / steady; t0 = grid ramp + tail + launch gap"}}
print(json.dumps(out, indent=1))
if len(sys.argv) > 2:
    json.dump(out, open(sys.argv[2], "w"), indent=1)
