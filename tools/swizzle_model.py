#!/usr/bin/env python3
"""LDS bank-conflict model of the generic f32 CFFT kernel (cfft_f32_core.hpp) and a search for
linear (XOR) workgroup-image swizzles.  EXPERIMENT, NOT DEPLOYED: the searched swizzles cut the
modelled conflict cycles (e.g. N=4096 3456 -> 2816 with the write banking below) but measured
10-30 % SLOWER (profiles/r01/swizzle_experiment.txt): an XOR with a per-access constant cannot
be folded into the ds_read/ds_write offset field, so every access pays a VALU op, and the kernel
is VALU- rather than LDS-bound.  The shipped swizzle, i ^ (((i>>4)&15)<<1), leaves the stage
offsets additive.

Every ds_read_b64 / ds_write_b64 the kernel issues is listed as 64 image addresses (one
workgroup = 256 threads, TPB transforms of N complex = 4096 float2): the radix8by2 /
radix8by4 first pass, each radix-8 stage, the 16-B load scatter and the digit-reversed
gather.  Cost of one access = sum over its two 32-lane halves of the largest number of
distinct float2 addresses sharing a bank pair; reads (ds_read_b64): two 32-lane groups,
bank (a/4) mod 64; writes (ds_write_b64): four 16-lane groups, bank (a/4) mod 32
(MI355X_MICROARCH.md §LDS).  A swizzle is a ^ ((a>>s0)&m0) ^ ((a>>s1)&m1) ^ ((a>>s2)&m2), bits pulled only
from a >= 32 (bijective on aligned 32-blocks).  Usage: python tools/swizzle_model.py [--search]
"""
import sys

import numpy as np

CHOSEN = {16: [(5, 15), (2, 24)], 32: [(8, 31), (5, 27), (3, 20)], 64: [(2, 24), (5, 31), (6, 7)],
          128: [(5, 31), (3, 28), (6, 31)], 256: [(6, 20), (5, 15), (4, 30)], 512: [(3, 24), (5, 15), (6, 6)],
          1024: [(5, 7), (3, 24), (8, 1)], 2048: [(6, 31), (3, 28), (5, 1)], 4096: [(5, 9), (4, 30), (7, 31)]}


def plan(n):
    first = 2 if n in (16, 128, 1024) else 4 if n in (32, 256, 2048) else 1
    length = n // first
    return first, length, int(np.log2(length)) // 3


def f32_src(n, k):
    first, _, stages = plan(n)
    p, rem = np.zeros_like(k), n
    if first > 1:
        rem //= first
        p += (k % first) * rem
        k = k // first
    for _ in range(stages):
        rem >>= 3
        p += (k & 7) * rem
        k = k >> 3
    return p


def accesses(n):
    first, length, stages = plan(n)
    lpt, out = n // 16, []
    for w in range(4):
        tid = w * 64 + np.arange(64)
        t, lane = tid // lpt, tid % lpt
        base = t * n
        if first == 2:
            q, h = n // 4, n // 2
            for it in range(q // lpt):
                k = lane + it * lpt
                out += [("first", base + k + o) for o in (0, h, q, h + q)]
        elif first == 4:
            q, e = n // 4, n // 8
            for it in range(q // lpt):
                ww = lane + it * lpt
                k = np.where(ww <= e, ww, q - (ww - e))
                out += [("first", base + k + o) for o in (0, q, 2 * q, 3 * q)]
        for s in range(stages):
            n1 = length >> (3 * s)
            n2 = n1 >> 3
            for r in range((n // 8) // lpt):
                b = lane + r * lpt
                c, rr = b // (length // 8), b % (length // 8)
                j, qq = rr % n2, rr // n2
                bi = c * length + qq * n1 + j
                out += [(f"stage{s}", base + bi + m * n2) for m in range(8)]
    for w in range(32):
        e = 2 * (w * 64 + np.arange(64))
        t, k = e // n, e % n
        for h in (0, 1):
            out += [("load", t * n + k + h), ("gather", t * n + f32_src(n, k + h))]
    return out


def swizzle(terms):
    def f(a):
        h = np.zeros_like(a)
        for s, m in terms:
            h ^= (a >> s) & m
        return a ^ h
    return f


def cost(addr, write=False):
    c, g = 0, 16 if write else 32
    for k in range(0, 64, g):
        u = np.unique(addr[k:k + g])
        c += np.bincount(u % g, minlength=g).max()
    return c


def total(n, f):
    d = {}
    for name, a in accesses(n):
        rd = name != "load"
        wr = name != "gather"
        d[name] = d.get(name, 0) + (cost(f(a)) if rd else 0) + (cost(f(a), True) if wr else 0)
    return d


def search(n, rng, trials=20000):
    acc = accesses(n)
    best = None
    for _ in range(trials):
        terms = []
        for _ in range(3):
            s, m = int(rng.integers(1, 12)), int(rng.integers(1, 32))
            if (m & -m).bit_length() - 1 + s >= 5:
                terms.append((s, m))
        f = swizzle(terms)
        c = sum(sum(total(n, f).values()) for _ in [0])
        if best is None or c < best[0]:
            best = (c, terms)
    return best


if __name__ == "__main__":
    rng = np.random.default_rng(0)
    for n, terms in CHOSEN.items():
        ideal = sum((2 if nm != "load" else 0) + (4 if nm != "gather" else 0) for nm, _ in accesses(n))
        old = (lambda a: a ^ (((a >> 4) & 15) << 1)) if n >= 512 else (lambda a, n=n: a + a // n if n <= 64 else a)
        line = f"N={n:5d} conflict-free {ideal:5d}  chosen {sum(total(n, swizzle(terms)).values()):5d}  " \
               f"previous {sum(total(n, old).values()):5d}"
        if "--search" in sys.argv:
            line += f"  random-search {search(n, rng)}"
        print(line)
