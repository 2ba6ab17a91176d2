#!/usr/bin/env python3
"""Access-pattern model of the radix-16-pass fixed-point CFFT kernels (cfft_fixed_r16.hip):
for each N, the element index every lane touches in every pass, and a search for additive
LDS paddings s(e) = e + c1*(e >> k1) + c2*(e >> k2) (plus a per-transform slot stride) that are
bank-conflict free under the MI355X LDS banking of the instructions the kernels use
(MI355X_MICROARCH.md §LDS):
  q31 (8-B complex): ds_read2_b64 / ds_write_b64 / ds_write2_b64 -> 16-lane groups, bank =
                     dword mod 32, i.e. 16 complex slots;
  q15 (4-B complex): ds_read2_b32 / ds_write_b32 -> 32-lane groups, bank = dword mod 32.
Usage: fx_r16_plan.py [N ...]  -> prints the best paddings per N and type."""
import itertools
import sys


def rev(x, n):
    return int(format(x, "0%db" % n)[::-1], 2) if n else 0


def log2(x):
    return x.bit_length() - 1


def plan(N):
    by2 = log2(N) % 2 == 1
    M = N // 2 if by2 else N
    K = log2(M) // 2
    P = N // 16
    passes = []                      # list of functions t' -> list of 16 element indices
    if by2:
        passes.append(lambda tp: [tp + P * u for u in range(16)])
        s = 2
        half_threads = P // 2
    else:
        s = 1
        half_threads = P
    while s <= K:
        if s + 1 <= K:
            L = M // 4 ** (s - 1)
            d1, d2 = L // 4, L // 16
            last = s + 1 == K
            def f(tp, L=L, d1=d1, d2=d2, last=last):
                h, tq = (tp & 1, tp >> 1) if by2 else (0, tp)
                if last:
                    g = rev(tq, log2(M // 16))
                    return [h * M + 16 * g + a + 4 * b for a in range(4) for b in range(4)]
                g, j = tq // d2, tq % d2
                return [h * M + g * L + j + d2 * a + d1 * b for a in range(4) for b in range(4)]
            if not (s == 1 and not by2):
                passes.append(f)
            else:
                passes.append(lambda tp, d1=d1, d2=d2: [tp + d2 * a + d1 * b for a in range(4) for b in range(4)])
            s += 2
        else:
            def f1(tp):
                h, tq = (tp & 1, tp >> 1) if by2 else (0, tp)
                nb = log2(M // 4)
                return [h * M + 4 * rev(tq + half_threads * c, nb) + b for c in range(4) for b in range(4)]
            passes.append(f1)
            s += 1
    return dict(N=N, by2=by2, M=M, K=K, P=P, TPW=256 // P, passes=passes)


def check_cover(pl):
    for f in pl["passes"]:
        seen = sorted(e for tp in range(pl["P"]) for e in f(tp))
        assert seen == list(range(pl["N"])), (pl["N"], "pass does not cover")


def lane_elems(pl):
    """[pass][u] -> (transform index per lane, element index per lane) for the 256 lanes."""
    import numpy as np
    P = pl["P"]
    t = np.arange(256)
    w, tp = t // P, t % P
    out = []
    for f in pl["passes"]:
        E = np.array([f(x) for x in range(P)])          # [P][16]
        out.append([(w, E[tp, u]) for u in range(16)])
    return out


def conflicts(pl, pad, stride, q31, le=None, limit=None):
    """Extra LDS cycles per workgroup, summed over every pass's 16 accesses."""
    import numpy as np
    le = le or lane_elems(pl)
    grp = 16 if q31 else 32
    slots = 16 if q31 else 32
    tot = 0
    for ps in le:
        for w, e in ps:
            a = w * stride + pad(e)
            A = a.reshape(-1, grp)
            key = np.sort((A % slots) * (1 << 20) + A, axis=1)
            uniq = np.concatenate([np.ones((key.shape[0], 1), bool), np.diff(key, axis=1) != 0], axis=1)
            banks = key >> 20
            for r in range(A.shape[0]):
                c = np.bincount(banks[r][uniq[r]], minlength=slots).max()
                tot += c - 1
            if limit is not None and tot > limit:
                return tot
    return tot


def search(N, q31):
    pl = plan(N)
    check_cover(pl)
    le = lane_elems(pl)
    best = None
    ks = range(3, 11)
    for k1, k2 in itertools.combinations_with_replacement(ks, 2):
        for c1 in (0, 1, 2, 4, 8):
            for c2 in (0, 1, 2, 4, 8):
                if (k1 == k2 and c2) or (c1 == 0 and c2 == 0 and k1 != 3):
                    continue
                pad = lambda e, k1=k1, k2=k2, c1=c1, c2=c2: e + c1 * (e >> k1) + c2 * (e >> k2)
                size = int(pad(N - 1)) + 1
                for extra in (0, 1, 2, 4, 8, 16, 24, 32):
                    stride = size + extra
                    lim = best[0][0] if best else None
                    c = conflicts(pl, pad, stride, q31, le, lim)
                    key = (c, stride, c1 + c2)
                    if best is None or key < best[0]:
                        best = (key, dict(k1=k1, c1=c1, k2=k2, c2=c2, stride=stride))
                    if c == 0:
                        break
    return best


if __name__ == "__main__":
    for N in [int(a) for a in sys.argv[1:]] or [256, 512, 1024, 2048]:
        for q31 in (True, False):
            b = search(N, q31)
            print(N, "q31" if q31 else "q15", "conflict cycles/wave", b[0][0], "slots", b[0][1], b[1])
