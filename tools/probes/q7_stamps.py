"""Summarise the in-kernel barrier timestamps of the persistent ping-pong q7 GEMM
(tools/probes/q7_stamps.hip, built with -DMI355X_Q7_STAMP=1): per workgroup and wave group the
s_memtime stamps at every barrier; the intervals between consecutive barriers are the ping-pong
half-phases (one group's MFMA segment beside the other's read / DMA segment).

A build with -DMI355X_Q7_STAMP=2 (the 128-deep kernel only) writes, instead, per workgroup and
group the s_memtime ticks summed per loop segment (entries 3..7: L segment, epilogue, barrier after
L, MFMA segment, barrier after M); `--phases` prints their means per step.

usage: python tools/probes/q7_stamps.py [--phases] stamps.json [more.json ...]
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


def phases(path, steps=32):
    d = json.load(open(path))
    st = np.array(d["stamps"], dtype=np.int64)[:, :, :8]
    names = ["L_segment", "epilogue", "barrier_after_L", "mfma_segment", "barrier_after_M"]
    out = {"file": path, "launch_ms": d["ms"]}
    for g in (0, 1):
        m = st[:, g, :].mean(axis=0) / steps
        out[f"group{g}"] = {n: round(float(v)) for n, v in zip(names, m[3:8])}
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    ph = args and args[0] == "--phases"
    for p in args[1:] if ph else args:
        print(json.dumps(phases(p) if ph else summary(p)))
