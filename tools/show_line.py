#!/usr/bin/env python3
"""Print value / roofline fraction / bit-exactness of the last JSON line of a bench output.
Usage: show_line.py <file> [label]"""
import json
import sys

lines = [ln for ln in open(sys.argv[1]) if ln.startswith("{")]
d = json.loads(lines[-1])
r = d.get("roofline", {})
print(sys.argv[2] if len(sys.argv) > 2 else "", d.get("value"), d.get("unit"), r.get("frac"), r.get("avg_kernel_ms"),
      d.get("parity", {}).get("bit_exact"))
