"""Summarise the in-kernel barrier timestamps of the persistent ping-pong q7 GEMM
(tools/probes/q7_stamps.hip, built with -DMI355X_Q7_STAMP=1): per workgroup and wave group the
s_memtime stamps at every barrier; the intervals between consecutive barriers are the ping-pong
half-phases (one group's MFMA segment beside the other's read / DMA segment).

usage: python tools/probes/q7_stamps.py stamps.json [more.json ...]
"""
import json
import sys

import numpy as np


def summary(path):
    d = json.load(open(path))
    st = np.array(d["stamps"], dtype=np.int64)          # [workgroup][group][k]
    out = {"file": path, "launch_ms": d["ms"]}
    iv, span = [], []
    for w in range(st.shape[0]):
        s = st[w, 0]
        s = s[s > 0]
        if len(s) < 4:
            continue
        dd = np.diff(s)
        iv.append(dd[1:])                               # [0]: start -> prologue barrier
        span.append(s[-1] - s[0])
    iv = np.concatenate(iv)
    out["intervals"] = {"count": int(iv.size), "p10": float(np.percentile(iv, 10)),
                        "median": float(np.median(iv)), "p90": float(np.percentile(iv, 90)),
                        "mean": float(iv.mean())}
    out["long_intervals_over_2k"] = int((iv > 2000).sum())
    out["wave_span_median"] = float(np.median(span))
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(json.dumps(summary(p)))
