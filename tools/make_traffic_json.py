#!/usr/bin/env python3
"""Collect tools/profile_pmc.sh results into profiles/<round>/ and profiles/pmc_traffic.json.

traffic per launch = FETCH_SIZE*1024*2 (gfx950 reports half of wide coalesced reads;
MI355X_MICROARCH.md §HBM; cross-checked against TCC_EA0_RDREQ*128 and against torch's copy
kernel on a known 8 GiB byte count, tools/profile_calibrate.sh) + WRITE_SIZE*1024.
Usage: make_traffic_json.py <round> <workload>=<prof_dir>:<kernel-substring> ...
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rnd = sys.argv[1]
    dest = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(dest, exist_ok=True)
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    traffic = json.load(open(path)) if os.path.exists(path) else {}
    for spec in sys.argv[2:]:
        wl, rest = spec.split("=")
        pdir, ksub = rest.split(":")
        out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), pdir, ksub],
                             capture_output=True, text=True, check=True).stdout
        summ = json.loads(out)
        with open(os.path.join(dest, f"{wl}_pmc_summary.json"), "w") as f:
            f.write(out)
        stats = os.path.join(pdir, "trace", "run_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(dest, f"{wl}_kernel_stats.csv"))
        traffic[wl] = {"hbm_bytes_per_launch": round(summ["fetch_bytes_raw"] * 2 + summ["write_bytes"]),
                       "read_bytes": round(summ["fetch_bytes_raw"] * 2), "write_bytes": round(summ["write_bytes"]),
                       "kernel": ksub, "round": rnd, "source": f"profiles/{rnd}/{wl}_pmc_summary.json"}
    with open(path, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    print(json.dumps(traffic, indent=1))


if __name__ == "__main__":
    main()
