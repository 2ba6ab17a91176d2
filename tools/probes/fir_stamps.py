"""Summarise tools/probes/fir_stamps.hip: median s_memtime ticks of each phase of an item (wave 0
of workgroups 0-63, items 2-63: past the warm-up).
usage: python tools/probes/fir_stamps.py stamps.json"""
import json
import sys

import numpy as np

NAMES = ["barrier A (prev. item's reads)", "stage (incl. the wait for this item's loads)", "barrier B",
         "issue next loads", "MFMA + output arithmetic", "stores", "to next loop top"]

d = json.load(open(sys.argv[1]))
st = np.array(d["stamps"], dtype=np.int64)             # [wg][item][event]
ph = []
for w in range(st.shape[0]):
    for k in range(2, st.shape[1] - 1):
        e = st[w, k]
        if e[0] == 0 or e[6] == 0 or st[w, k + 1, 0] == 0:
            continue
        ph.append([e[1] - e[0], e[2] - e[1], e[3] - e[2], e[4] - e[3], e[5] - e[4], e[6] - e[5], st[w, k + 1, 0] - e[6]])
ph = np.array(ph)
out = {"launch_ms": d["ms"], "items": int(len(ph)), "median_item_ticks": float(np.median(ph.sum(1)))}
out["phases_median"] = {n: float(np.median(ph[:, i])) for i, n in enumerate(NAMES)}
out["phases_mean"] = {n: round(float(ph[:, i].mean()), 1) for i, n in enumerate(NAMES)}
print(json.dumps(out, indent=1))
