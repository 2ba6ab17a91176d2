"""Probe: numpy models of the reference's conv / correlate / partial-conv variants, checked
against the reference build (oracle/_ref) over many length pairs and input distributions.

It pins down the arithmetic contract the GPU kernels restate (DESIGN.md §conv family):
* exact variants (f32, q15, q31, partial): the full overlap sum, pSrcA... ascending;
* fast q31: sum of floor(x*y / 2^32) mod 2^32, output << 1;
* fast q15: sum of x*y mod 2^32 plus +1 per single-sample __SMLAD with both operands
  negative (none.h:455-463 extracts the high halfword of a sign-extended q15 as -1), output
  (q15)(sum >> 15).
Run: python tools/probes/conv_family_model.py   (needs oracle/_ref/libcmsisdsp_ref.so)
"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
lib = C.CDLL(os.path.join(ROOT, "oracle", "_ref", "libcmsisdsp_ref.so"))
DT = {"f32": np.float32, "q15": np.int16, "q31": np.int32}


def ref_call(name, kind, a, b, out_len, *extra):
    a = np.ascontiguousarray(a, DT[kind])
    b = np.ascontiguousarray(b, DT[kind])
    y = np.full(out_len, 0x5A5A if kind != "f32" else 7.0, dtype=DT[kind])
    f = getattr(lib, name)
    f.restype = C.c_int
    st = f(C.c_void_p(a.ctypes.data), C.c_uint32(len(a)), C.c_void_p(b.ctypes.data), C.c_uint32(len(b)),
           C.c_void_p(y.ctypes.data), *[C.c_uint32(e) for e in extra])
    return y, st


def full_sums(x, h, acc):
    """v[n] = sum_k x[k] * h[n-k] in the accumulator semantics `acc`."""
    A, B = len(x), len(h)
    out = []
    for n in range(A + B - 1):
        k0, k1 = max(0, n - B + 1), min(n, A - 1)
        out.append(acc(x[k0:k1 + 1], h[n - np.arange(k0, k1 + 1)], n, k0, k1))
    return out


def q15_fast_singles_conv(A, B, n):
    """k range [s, e] of single-sample __SMLAD MACs for output n of arm_conv_fast_q15
    (x = the longer input, A >= B)."""
    if n <= B - 2:                                  # stage 1: count = n + 1
        c = n + 1
        return n + 1 - c % 4, n
    if n <= A - 1:
        return 1, 0                                 # stage 2: none
    i = n - A
    bs3 = B - 1 - i
    if i < (B - 1) // 4:
        return A - bs3 % 4, A - 1
    return n - B + 1, A - 1


def q15_fast_singles_corr(A, B, n):
    if n <= B - 2:
        c = n + 1
        return n + 1 - c % 4, n
    if n <= A - 1:
        return 1, 0
    c = A + B - 1 - n
    return A - c % 4, A - 1


def model(fn, kind, a, b, first=0, num=0):
    A0, B0 = len(a), len(b)
    a = np.asarray(a).astype(np.int64) if kind != "f32" else np.asarray(a, np.float32)
    b = np.asarray(b).astype(np.int64) if kind != "f32" else np.asarray(b, np.float32)
    corr = fn.startswith("correlate")
    fast = "fast" in fn
    # x = the input summed in ascending index
    if corr:
        x, s = (a, b) if A0 >= B0 else (b, a)
        h = s[::-1]
    elif fast:
        x, h = (a, b) if A0 >= B0 else (b, a)
    else:
        x, h = a, b
    A, B = len(x), len(h)

    def wrap(v, bits):
        v %= 2**bits
        return v - 2**bits if v >= 2**(bits - 1) else v

    def acc(xs, hs, n, k0, k1):
        if kind == "f32":
            s = np.float32(0)
            for p, q in zip(xs, hs):
                s = np.float32(s + np.float32(p * q))
            return s
        prods = [int(p) * int(q) for p, q in zip(xs, hs)]
        if not fast:
            s = wrap(sum(prods), 64)
            if kind == "q15":
                return max(-32768, min(32767, wrap(s >> 15, 32)))
            return wrap(s >> 31, 32)
        if kind == "q31":
            return wrap(sum(p >> 32 for p in prods) << 1, 32)
        s = sum(prods)
        lo, hi = (q15_fast_singles_corr if corr else q15_fast_singles_conv)(A, B, n)
        for k in range(lo, hi + 1):
            s += int(x[k] < 0 and h[n - k] < 0)
        return wrap(wrap(s, 32) >> 15, 16)

    dt = DT[kind]
    v = np.array(full_sums(x, h, acc), dtype=np.float32 if kind == "f32" else np.int64).astype(dt)
    if corr:
        L = 2 * max(A0, B0) - 1
        y = np.full(L, 0x5A5A if kind != "f32" else 7.0, dtype=dt)
        if A0 >= B0:
            y[A0 - B0:A0 - B0 + len(v)] = v
        else:
            y[:len(v)] = v[::-1]
        return y
    if fn.startswith("conv_partial"):
        y = np.full(A0 + B0 - 1, 0x5A5A if kind != "f32" else 7.0, dtype=dt)
        y[first:first + num] = v[first:first + num]
        return y
    return v


def rand(kind, n, rng, dist):
    if kind == "f32":
        return rng.uniform(-1, 1, n).astype(np.float32)
    info = np.iinfo(DT[kind])
    if dist == "full":
        return rng.integers(info.min, info.max, n, endpoint=True).astype(DT[kind])
    if dist == "neg":
        return rng.integers(info.min, 0, n).astype(DT[kind])
    return (rng.integers(-2**(info.bits - 4), 2**(info.bits - 4), n)).astype(DT[kind])


def main():
    rng = np.random.default_rng(1)
    fails = 0
    cases = [(a, b) for a in (1, 2, 3, 4, 5, 7, 8, 9, 13, 16, 17, 33) for b in (1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 13, 17, 33)]
    fns = sys.argv[1:] or ["correlate_f32", "correlate_q15", "correlate_q31", "correlate_fast_q31", "conv_fast_q31",
                           "conv_fast_q15", "correlate_fast_q15", "conv_partial_f32", "conv_partial_q15",
                           "conv_partial_q31", "conv_partial_fast_q31", "conv_partial_fast_q15"]
    for fn in fns:
        kind = fn[-3:]
        bad = 0
        for (la, lb) in cases:
            for dist in (("small", "full", "neg") if kind != "f32" else ("u",)):
                a, b = rand(kind, la, rng, dist), rand(kind, lb, rng, dist)
                if fn.startswith("conv_partial"):
                    L = la + lb - 1
                    for first in sorted({0, 1, 2, 3, lb - 1, lb, la - 1, la, L // 2, L - 3, L - 1}):
                        if not 0 <= first < L:
                            continue
                        for num in sorted({1, 2, 3, 4, 5, L - first, (L - first) // 2}):
                            if num < 1 or first + num > L:
                                continue
                            r, st = ref_call("arm_" + fn, kind, a, b, L, first, num)
                            m = model(fn, kind, a, b, first, num)
                            if r.tobytes() != m.tobytes() or st != 0:
                                bad += 1
                                if bad <= 3:
                                    print(fn, la, lb, dist, first, num, "ref", r, "model", m)
                    continue
                L = 2 * max(la, lb) - 1 if fn.startswith("correlate") else la + lb - 1
                r, _ = ref_call("arm_" + fn, kind, a, b, L)
                m = model(fn, kind, a, b)
                if r.tobytes() != m.tobytes():
                    bad += 1
                    if bad <= 3:
                        print(fn, la, lb, dist, "ref", r, "model", m)
        print(f"{fn:24s} mismatching cases: {bad}")
        fails += bad
    return fails


if __name__ == "__main__":
    sys.exit(1 if main() else 0)
