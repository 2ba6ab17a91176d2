"""Per-kernel summary of a rocprofv3 rocpd database (run_results.db): dispatch count and
average / min duration of the largest-grid dispatches, for kernels matching a substring."""
import sqlite3
import sys
from collections import defaultdict


def summary(db, sub=""):
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, duration from kernels").fetchall()
    d = defaultdict(list)
    for name, gx, dur in rows:
        if sub in name:
            d[(name.split("(")[0][-60:], gx)].append(dur)
    return {k: (len(v), sum(v) / len(v) / 1e6, min(v) / 1e6) for k, v in d.items()}


if __name__ == "__main__":
    for k, (n, avg, mn) in sorted(summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "").items()):
        print(f"{k[0]:62s} grid {k[1]:>9d}  n {n:3d}  avg {avg:.4f} ms  min {mn:.4f} ms")
