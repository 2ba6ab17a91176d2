"""Condensed view of one kernel in a device .s file: waits, memory ops, barriers and branch
labels, with runs of VALU arithmetic collapsed into counts.
Usage: python tools/isa_summary.py file.s <kernel-name-substring> [max_lines]"""
import sys

path, key = sys.argv[1], sys.argv[2]
limit = int(sys.argv[3]) if len(sys.argv) > 3 else 300
lines = open(path).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l.split(":")[0] and l.rstrip().endswith(
    l.split(":")[0].split()[-1] + ":") or (l.startswith("_Z") and key in l and ": ;" in l))
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
out, cnt = [], 0
for l in lines[start:end]:
    t = l.strip()
    if t.startswith(("v_",)) and not t.startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
        cnt += 1
        continue
    if cnt:
        out.append(f"    [{cnt} valu]")
        cnt = 0
    if t.startswith(("s_waitcnt", "s_load", "s_buffer_load", "ds_", "s_cbranch", "s_branch", ".LBB", "s_barrier",
                     "buffer_", "global_", "s_sleep", "s_endpgm")):
        out.append(t.split(";")[0].rstrip())
print("\n".join(out[:limit]))
