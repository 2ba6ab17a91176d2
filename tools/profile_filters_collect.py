#!/usr/bin/env python3
"""Collect tools/profile_filters.sh output into profiles/<round>/filters_<tag>/: per workload the
rocprofv3 --stats summary, the dominant kernel's trace average over its timed launches (the last
10 of its largest grid: bench_filters.py times 10 steps) next to the bench line's HIP-event
average, and HBM bytes per launch from the FETCH_SIZE / WRITE_SIZE passes (read = 2 x FETCH_SIZE
KiB, the gfx950 correction in MI355X_MICROARCH.md; write = WRITE_SIZE KiB) against the
algorithmic bytes (input + output words; histories are < 1 %).
Usage: profile_filters_collect.py <round> <tag>"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from profile_collect import bench_line, pmc_summary, trace_summary  # noqa: E402

KERNEL = {"fir_q7": "fir_q7_kernel", "fir_decimate_f32_m4": "fir_f32_kernel",
          "fir_decimate_q15_m4": "fir_decimate_kernel", "fir_interpolate_f32_l4": "fir_interp_phases_kernel",
          "fir_sparse_f32": "fir_sparse_lds_kernel", "fir_sparse_q7": "fir_sparse_lds_kernel",
          "fir_lattice_f32": "fir_lattice_kernel", "fir_lattice_q31": "fir_lattice_kernel"}
ESZ = {"f32": 4, "q31": 4, "q15": 2, "q7": 1}


def main():
    rnd, tag = sys.argv[1], sys.argv[2]
    src = os.path.join(ROOT, "gpurun_out", f"prof_filters_{tag}")
    dest_root = os.path.join(ROOT, "profiles", rnd, f"filters_{tag}")
    index = {}
    for name in sorted(os.listdir(src)):
        d = os.path.join(src, name)
        ksub = KERNEL[name]
        line = bench_line(os.path.join(d, "bench.json"))
        tr = trace_summary(d, 10)
        dom = max((k for k in tr if ksub in k), key=lambda k: tr[k]["timed_avg_ms"] * tr[k]["timed_dispatches"])
        rec = {"workload": name, "kernel": dom, "trace_timed_avg_ms": tr[dom]["timed_avg_ms"],
               "timed_grid": tr[dom]["timed_grid"], "bench_hip_event_avg_ms": line["avg_kernel_ms"],
               "bench": line}
        rec["trace_over_hip_event"] = rec["trace_timed_avg_ms"] / line["avg_kernel_ms"]
        pm = pmc_summary(d, ksub)
        if pm:
            c, _ = pm
            kind = line["function"].split("_")[-1]
            algo = line["batch"] * (line["blockSize"] + line["output_gsamples_per_s"] / line["input_gsamples_per_s"]
                                    * line["blockSize"]) * ESZ[kind]
            rec["read_bytes"] = c.get("FETCH_SIZE", 0) * 1024 * 2
            rec["write_bytes"] = c.get("WRITE_SIZE", 0) * 1024
            rec["hbm_bytes_per_launch"] = rec["read_bytes"] + rec["write_bytes"]
            rec["algorithmic_bytes_per_launch"] = algo
            rec["traffic_over_algorithmic"] = rec["hbm_bytes_per_launch"] / algo
        dest = os.path.join(dest_root, name)
        os.makedirs(dest, exist_ok=True)
        for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(dest, "run_kernel_stats.csv"))
        json.dump(rec, open(os.path.join(dest, "summary.json"), "w"), indent=1)
        index[name] = {k: rec.get(k) for k in ("kernel", "trace_timed_avg_ms", "bench_hip_event_avg_ms",
                                               "trace_over_hip_event", "hbm_bytes_per_launch",
                                               "traffic_over_algorithmic")}
    json.dump(index, open(os.path.join(dest_root, "INDEX.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(index, indent=1))


if __name__ == "__main__":
    main()
