"""Static VALU mix of one kernel's hottest loop in a device .s file (hipcc -S --cuda-device-only),
for the `valu_issue` blocks of the bench lines and DESIGN §4.

Every instruction of the blocks LLVM tags as one loop ("; =>This Inner Loop Header" / "in Loop:
Header=...") is classed by its issue rate on gfx950, from the op-rate probe
(profiles/r04/probes/op_rate.txt: 56-66 T lane-instr/s for VOP1/VOP2 integer and f32 ops, 34-38 for
VOP3 / VOP3P / dot / 64-bit multiply-add -- i.e. 2 and 4 cycles per wave64 instruction):
  full  -- 2 cycles per wave-instruction (VOP1 / VOP2, e32 encodings, v_fmac / v_mul_f32 ...);
  half  -- 4 cycles (VOP3 three-operand integer ops, v_pk_*, v_dot*, v_mad_*, v_mul_hi / lo,
           v_perm / v_alignbit / v_bfe / v_med3 / cvt_pk ...);
  trans -- 8 cycles (v_exp / v_log / v_rcp / v_rsq / v_sqrt / v_sin / v_cos);
  mfma  -- counted apart.
usage: python tools/valu_mix.py file.s <kernel-substring> [--loop LABEL]
prints JSON: per-class counts of the loop with the most VALU instructions (or --loop), and the
issue cycles per iteration per wave (full 2, half 4, trans 8).
"""
import json
import re
import sys

HALF_PREFIX = ("v_pk_", "v_dot", "v_mad", "v_mul_hi", "v_mul_lo", "v_perm", "v_alignbit", "v_alignbyte", "v_bfe",
               "v_bfi", "v_med3", "v_min3", "v_max3", "v_cvt_pk", "v_lshl_add", "v_add_lshl", "v_lshl_or", "v_and_or",
               "v_or3", "v_xad", "v_add3", "v_sad", "v_mqsad", "v_lerp", "v_fma_f64", "v_add_f64", "v_mul_f64",
               "v_div", "v_ldexp", "v_cvt_pkrtz", "v_mul_u32_u24", "v_mad_u32", "v_lshlrev_b64", "v_lshrrev_b64",
               "v_ashrrev_i64", "v_lshl_add_u64", "v_mov_b64", "v_sat_pk", "v_permlane")
TRANS_PREFIX = ("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")


def classify(op, line):
    if op.startswith("v_mfma") or op.startswith("v_smfmac"):
        return "mfma"
    if op.startswith(TRANS_PREFIX):
        return "trans"
    if op.startswith(("v_readfirstlane", "v_readlane", "v_writelane", "v_accvgpr")):
        return "full"
    if op.startswith(HALF_PREFIX) or op.endswith("_e64"):
        return "half"
    return "full"


def kernel_lines(path, key):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and key in l.split()[0] and l.split()[0].endswith(":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def loops(body):
    """label -> list of instruction lines of the blocks belonging to that loop header."""
    out, cur = {}, None
    for l in body:
        m = re.match(r"^(\.LBB\w+):.*(Loop Header|in Loop: Header=(\w+))", l)
        if m:
            cur = m.group(1) if "Loop Header" in l and "in Loop" not in l else "." + "LBB" + m.group(3)[2:]
            out.setdefault(cur, [])
            continue
        if re.match(r"^\.LBB\w+:", l) or re.match(r"^; %bb", l):
            mm = re.search(r"in Loop: Header=(\w+)", l)
            cur = ("." + "LBB" + mm.group(1)[2:]) if mm else None
            if cur:
                out.setdefault(cur, [])   # a loop block laid out before its header
            continue
        if cur and l.startswith("\t") and not l.strip().startswith((";", ".")):
            out[cur].append(l.strip())
    return out


def mix(instrs):
    c = {"full": 0, "half": 0, "trans": 0, "mfma": 0, "lds": 0, "vmem": 0, "salu": 0}
    for t in instrs:
        op = t.split()[0]
        if op.startswith("v_"):
            c[classify(op, t)] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    c["issue_cycles_per_wave"] = 2 * c["full"] + 4 * c["half"] + 8 * c["trans"]
    return c


if __name__ == "__main__":
    path, key = sys.argv[1], sys.argv[2]
    want = sys.argv[sys.argv.index("--loop") + 1] if "--loop" in sys.argv else None
    body = kernel_lines(path, key)
    ls = loops(body)
    whole = mix([l.strip() for l in body if l.startswith("\t")])
    if ls:
        pick = want or max(ls, key=lambda k: sum(1 for t in ls[k] if t.startswith("v_")))
        out = {"kernel": key, "loop": pick, "loop_mix": mix(ls[pick]), "whole_kernel_mix": whole}
    else:
        out = {"kernel": key, "loop": None, "whole_kernel_mix": whole}
    print(json.dumps(out))
