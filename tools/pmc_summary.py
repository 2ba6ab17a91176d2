#!/usr/bin/env python3
"""Summarise tools/profile_pmc.sh output: per-dispatch averages of every counter for the
dominant kernel of a workload, and the HBM traffic per launch.

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE under-reports wide coalesced
reads by 2x (MI355X_MICROARCH.md §HBM), so the read side is also derived from
TCC_EA0_RDREQ (each request = 128 B on gfx950, tallied by FETCH_SIZE as 64 B) and the
two estimates are reported side by side.  Usage: pmc_summary.py <prof_dir> <kernel-substring>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def read_counters(d, ksub):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if ksub not in row.get("Kernel_Name", ""):
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        for (disp, name), v in per.items():
            vals[name].append(v)
    # average over the timed (large) dispatches only: the bench also launches the kernel on
    # a 64-item parity batch, which would otherwise pull every average down
    out = {}
    for k, v in vals.items():
        if v:
            big = [x for x in v if x >= 0.5 * max(v)] if max(v) > 0 else v
            out[k] = sum(big) / len(big)
    return out


def kernel_time(d, ksub):
    durs = []
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if ksub in row["Kernel_Name"]:
                durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    return durs


def main():
    d, ksub = sys.argv[1], sys.argv[2]
    c = read_counters(d, ksub)
    durs = kernel_time(d, ksub)
    big = [x for x in durs if x > 0.5 * max(durs)] if durs else []
    out = {"kernel": ksub, "dispatches": len(durs), "avg_ns_large_dispatches": (sum(big) / len(big)) if big else None,
           "counters_per_dispatch": c}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        out["fetch_bytes_raw"] = c["FETCH_SIZE"] * 1024
        out["write_bytes"] = c["WRITE_SIZE"] * 1024
    if "TCC_EA0_RDREQ_sum" in c:
        out["read_bytes_from_rdreq_x128"] = c["TCC_EA0_RDREQ_sum"] * 128
    if "TCC_EA0_WRREQ_sum" in c:
        out["write_bytes_from_wrreq_x64"] = c["TCC_EA0_WRREQ_sum"] * 64
    if "GRBM_GUI_ACTIVE" in c and big:
        out["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8 / out["avg_ns_large_dispatches"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
