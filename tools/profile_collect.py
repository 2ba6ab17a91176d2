#!/usr/bin/env python3
"""Collect tools/profile_round.sh output into profiles/<round>/<name>/ and
profiles/pmc_traffic.json.

Per workload:
  * kernel_trace.json — every kernel's dispatches from the --kernel-trace pass, averaged
    over the TIMED launches only (the dispatches with the kernel's largest grid: bench.py
    also launches it on small parity batches), next to the bench line's live HIP-event
    average of the same run (agreement ratio);
  * pmc.json — per-dispatch counter averages of the dominant kernel over its largest-grid
    dispatches, HBM bytes per launch (read = 2 x FETCH_SIZE: gfx950 tallies wide coalesced
    reads at half, MI355X_MICROARCH.md §HBM, cross-checked with TCC_EA0_RDREQ x 128; write
    = WRITE_SIZE), the effective clock (GRBM_GUI_ACTIVE per XCD over the kernel time) and,
    for MFMA kernels, MFMA busy cycles as a fraction of the SIMD cycles of the launch;
  * run_kernel_stats.csv — rocprofv3's own --stats summary (all dispatches);
  * for names whose spec lists source units, a valu_issue record: SQ_INSTS_VALU per launch of each
    kernel times its issue cycles per VALU instruction, weighted by the instruction classes of
    that kernel's hottest loop in its device assembly (tools/valu_mix.py on
    `make -C cmsis-dsp_amd build/<unit>.s`; full rate 2, half rate 4, transcendental 8 cycles per
    wave64 instruction per SIMD, profiles/r04/probes/op_rate.txt; MFMA issue counted 0).
pmc_traffic.json keys: the profile name; bench.py uses a record only when its recorded
bench config equals the line's config.
Usage: profile_collect.py <round> [name ...]
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from profile_specs import SPECS  # noqa: E402
import valu_mix  # noqa: E402

N_XCD, N_SIMD = 8, 1024


def _grid(row):
    if "Grid_Size" in row and row["Grid_Size"]:
        return int(row["Grid_Size"])
    return int(row.get("Grid_Size_X", 0) or 0) * int(row.get("Grid_Size_Y", 1) or 1) * int(row.get("Grid_Size_Z", 1) or 1)


def bench_line(path):
    try:
        for ln in open(path):
            if ln.startswith("{"):
                return json.loads(ln)
    except OSError:
        pass
    return None


def trace_summary(d, steps=None):
    """Per kernel: the largest-grid dispatches; with `steps` (the bench line's timed step
    count) only the LAST `steps` of them -- the timed region, after warmup and clock-settle
    launches of the same grid."""
    ks = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            t0, t1 = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
            ks[row["Kernel_Name"]].append((_grid(row), t1 - t0, t0))
    out = {}
    for k, v in ks.items():
        g = max(x[0] for x in v)
        big = sorted((x for x in v if x[0] == g), key=lambda x: x[2])
        timed = [x[1] for x in (big[-steps:] if steps and len(big) >= steps else big)]
        out[k] = {"dispatches": len(v), "largest_grid_dispatches": len(big), "timed_dispatches": len(timed),
                  "timed_grid": g, "timed_avg_ms": sum(timed) / len(timed) * 1e-6,
                  "largest_grid_avg_ms": sum(x[1] for x in big) / len(big) * 1e-6,
                  "all_avg_ms": sum(x[1] for x in v) / len(v) * 1e-6}
    return out


def merged_timed(d, sub, steps):
    """Mean duration (ms) of the last `steps` largest-grid dispatches of ALL kernels whose name
    contains `sub`, in dispatch order: the timed region when one step alternates template
    instances (configs[3]: forward / inverse), which the per-kernel `steps` cut would mix with
    warmup dispatches."""
    v = []
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if sub in row["Kernel_Name"]:
                v.append((_grid(row), int(row["End_Timestamp"]) - int(row["Start_Timestamp"]), int(row["Start_Timestamp"])))
    if not v or not steps:
        return None
    g = max(x[0] for x in v)
    big = sorted((x for x in v if x[0] == g), key=lambda x: x[2])[-steps:]
    return sum(x[1] for x in big) / len(big) * 1e-6


def pmc_summary(d, ksub):
    """Per-dispatch counter averages of the kernel(s) matching ksub; "a|b" sums the kernels of a
    multi-launch step (e.g. the MFCC front-end CFFT + post), each averaged over its timed grid."""
    if "|" in ksub:
        parts = [pmc_summary(d, k) for k in ksub.split("|")]
        if any(x is None for x in parts):
            return None
        tot = defaultdict(float)
        for c, _ in parts:
            for name, v in c.items():
                tot[name] += v
        return dict(tot), max(g for _, g in parts)
    per = defaultdict(lambda: defaultdict(float))     # (pass, dispatch) -> counter -> value
    grids = {}
    for f in glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        tag = os.path.relpath(f, d).split(os.sep)[0]
        for row in csv.DictReader(open(f)):
            if ksub not in row.get("Kernel_Name", ""):
                continue
            key = (tag, row["Dispatch_Id"])
            grids[key] = _grid(row)
            per[key][row["Counter_Name"]] += float(row["Counter_Value"])
    if not per:
        return None
    gmax = max(grids.values())
    acc = defaultdict(list)
    for key, cs in per.items():
        if grids[key] == gmax:
            for name, v in cs.items():
                acc[name].append(v)
    return {name: sum(v) / len(v) for name, v in acc.items()}, gmax


_ASM = {}


def kernel_asm(unit, kernel_name):
    """(mangled symbol, body lines) of the kernel whose demangled name (as the trace prints it)
    is kernel_name, from cmsis-dsp_amd/build/<unit>.s (built on demand)."""
    if unit not in _ASM:
        path = os.path.join(ROOT, "cmsis-dsp_amd", "build", f"{unit}.s")
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "cmsis-dsp_amd"), f"build/{unit}.s"], check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        syms = [l.split(":")[0] for l in open(path) if l.startswith("_Z") and ":" in l.split()[0]]
        dem = subprocess.run(["c++filt"], input="\n".join(syms), capture_output=True, text=True, check=True).stdout
        _ASM[unit] = (path, dict(zip(dem.strip().split("\n"), syms)))
    path, table = _ASM[unit]
    sym = table.get(kernel_name)
    return (sym, valu_mix.kernel_lines(path, sym)) if sym else (None, None)


def valu_issue(d, ksub, units, tr):
    """Issue cycles of the VALU instructions one launch executes (see the module docstring)."""
    parts, uparts = ksub.split("|"), units.split("|")
    out = {"by_kernel": {}, "valu_insts_per_launch": 0.0, "issue_cycles_per_launch": 0.0,
           "weighting": "hottest-loop instruction classes of the kernel's device assembly: full 2, half 4, "
                        "trans 8 cycles per wave64 VALU instruction, MFMA 0 (op_rate.txt)"}
    for part, unit in zip(parts, uparts):
        pm = pmc_summary(d, part)
        cand = [k for k in tr if part in k]
        if not pm or "SQ_INSTS_VALU" not in pm[0] or not cand:
            return None
        kname = max(cand, key=lambda k: tr[k]["timed_avg_ms"] * tr[k]["timed_dispatches"])
        sym, body = kernel_asm(unit, kname)
        if not body:
            return None
        ls = valu_mix.loops(body)
        whole = valu_mix.mix([l.strip() for l in body if l.startswith("\t")])
        if ls:
            pick = max(ls, key=lambda k: sum(1 for t in ls[k] if t.startswith("v_")))
            mx = valu_mix.mix(ls[pick])
        else:
            pick, mx = None, whole
        nv = mx["full"] + mx["half"] + mx["trans"] + mx["mfma"]
        cpi = mx["issue_cycles_per_wave"] / nv if nv else 2.0
        insts = pm[0]["SQ_INSTS_VALU"]
        out["by_kernel"][kname] = {"symbol": sym, "unit": unit, "loop": pick, "loop_mix": mx,
                                   "whole_kernel_mix": whole, "cycles_per_valu_inst": round(cpi, 4),
                                   "valu_insts_per_launch": insts, "issue_cycles_per_launch": insts * cpi}
        out["valu_insts_per_launch"] += insts
        out["issue_cycles_per_launch"] += insts * cpi
    return out


def main():
    rnd = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    names = sys.argv[2:] or sorted(n for n in os.listdir(src) if os.path.isdir(os.path.join(src, n)))
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    index = {}
    for name in names:
        d = os.path.join(src, name)
        ksub = SPECS[name][1]
        dest = os.path.join(ROOT, "profiles", rnd, name)
        os.makedirs(dest, exist_ok=True)
        line = bench_line(os.path.join(d, "bench_trace.json"))
        tr = trace_summary(d, line.get("steps") if line else None)
        dom = [k for k in tr if ksub.split("|")[0] in k]
        rec = {"name": name, "bench_args": SPECS[name][0], "dominant_kernel_substring": ksub, "kernels": tr,
               "bench_config": line.get("config") if line else None}
        if dom:
            k = max(dom, key=lambda k: tr[k]["timed_avg_ms"] * tr[k]["timed_dispatches"])
            rec["dominant_kernel"] = k
            rec["trace_timed_avg_ms"] = tr[k]["timed_avg_ms"]
            # multi-launch calls (e.g. arm_rfft_q31 = CFFT + split pass): the library's kernels
            # that ran once per timed step, summed, are what the bench's per-call events time
            steps = line.get("steps") if line else None
            pipe = [q for q in tr if "mi355x::" in q and steps and tr[q]["largest_grid_dispatches"] >= steps]
            rec["trace_pipeline_kernels"] = pipe
            rec["trace_pipeline_avg_ms"] = sum(tr[q]["timed_avg_ms"] for q in pipe) if pipe else None
            if len(dom) > 1 and steps:
                rec["trace_timed_avg_ms_all_instances"] = merged_timed(d, ksub.split("|")[0], steps)
            if line and line.get("roofline", {}).get("avg_kernel_ms"):
                rec["bench_hip_event_avg_ms"] = line["roofline"]["avg_kernel_ms"]
                rec["trace_over_hip_event"] = tr[k]["timed_avg_ms"] / line["roofline"]["avg_kernel_ms"]
                if rec.get("trace_timed_avg_ms_all_instances"):
                    rec["trace_all_instances_over_hip_event"] = (rec["trace_timed_avg_ms_all_instances"]
                                                                 / line["roofline"]["avg_kernel_ms"])
                if rec["trace_pipeline_avg_ms"]:
                    rec["pipeline_over_hip_event"] = rec["trace_pipeline_avg_ms"] / line["roofline"]["avg_kernel_ms"]
        for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(dest, "run_kernel_stats.csv"))
        json.dump(rec, open(os.path.join(dest, "kernel_trace.json"), "w"), indent=1)
        pm = pmc_summary(d, ksub)
        if pm:
            c, gmax = pm
            ms = rec.get("trace_pipeline_avg_ms") if "|" in ksub else rec.get("trace_timed_avg_ms")
            p = {"kernel_substring": ksub, "grid": gmax, "counters_per_dispatch": c}
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                p["read_bytes"] = c["FETCH_SIZE"] * 1024 * 2
                p["write_bytes"] = c["WRITE_SIZE"] * 1024
                p["hbm_bytes_per_launch"] = p["read_bytes"] + p["write_bytes"]
            if "TCC_EA0_RDREQ_sum" in c:
                p["read_bytes_from_rdreq_x128"] = c["TCC_EA0_RDREQ_sum"] * 128
            if "GRBM_GUI_ACTIVE" in c and ms:
                p["effective_clock_ghz"] = c["GRBM_GUI_ACTIVE"] / N_XCD / (ms * 1e6)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c and ms and "effective_clock_ghz" in p:
                simd_cycles = N_SIMD * ms * 1e6 * p["effective_clock_ghz"]
                p["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
            if line and line.get("roofline", {}).get("algorithmic_bytes_per_launch") and "hbm_bytes_per_launch" in p:
                p["traffic_over_algorithmic"] = p["hbm_bytes_per_launch"] / line["roofline"]["algorithmic_bytes_per_launch"]
            units = SPECS[name][2] if len(SPECS[name]) > 2 else ""
            if units:
                vi = valu_issue(d, ksub, units, tr)
                if vi:
                    p["valu_issue"] = vi
            json.dump(p, open(os.path.join(dest, "pmc.json"), "w"), indent=1)
            rec["pmc"] = {k: v for k, v in p.items() if k != "counters_per_dispatch"}
            if "hbm_bytes_per_launch" in p or "mfma_busy_frac" in p:
                traffic[name] = {"hbm_bytes_per_launch": round(p.get("hbm_bytes_per_launch", 0)) or None,
                                 "read_bytes": round(p.get("read_bytes", 0)), "write_bytes": round(p.get("write_bytes", 0)),
                                 "mfma_busy_frac": p.get("mfma_busy_frac"), "kernel": rec.get("dominant_kernel", ksub),
                                 "valu_insts_per_launch": p.get("valu_issue", {}).get("valu_insts_per_launch"),
                                 "valu_issue_cycles_per_launch": p.get("valu_issue", {}).get("issue_cycles_per_launch"),
                                 "avg_kernel_ms_trace": ms, "bench_config": rec["bench_config"], "round": rnd,
                                 "source": f"profiles/{rnd}/{name}/pmc.json"}
        index[name] = {k: rec.get(k) for k in ("dominant_kernel", "trace_timed_avg_ms", "bench_hip_event_avg_ms",
                                               "trace_over_hip_event", "trace_timed_avg_ms_all_instances",
                                               "trace_all_instances_over_hip_event", "trace_pipeline_avg_ms",
                                               "pipeline_over_hip_event")}
        index[name].update({k: rec.get("pmc", {}).get(k) for k in ("hbm_bytes_per_launch", "traffic_over_algorithmic",
                                                                   "effective_clock_ghz", "mfma_busy_frac")})
    json.dump(traffic, open(tpath, "w"), indent=1, sort_keys=True)
    ipath = os.path.join(ROOT, "profiles", rnd, "INDEX.json")
    old = json.load(open(ipath)) if os.path.exists(ipath) else {}
    old.update(index)
    json.dump(old, open(ipath, "w"), indent=1, sort_keys=True)
    print(json.dumps(index, indent=1))


if __name__ == "__main__":
    main()
