"""CPU: the oracle restatement is bit-identical to the reference scalar C (oracle/_ref,
compiled from /root/reference's own sources) on seeded inputs: every length, direction,
bit-reversal flag and input distribution, FIR streaming edge cases and mat_mult shapes."""
import numpy as np
import pytest

import refs

SIZES = [16, 32, 64, 128, 256, 512, 1024, 2048, 4096]


@pytest.mark.parametrize("kind", ["f32", "q31", "q15"])
@pytest.mark.parametrize("n", SIZES)
def test_cfft_oracle_equals_reference(oracle, ref, kind, n):
    dists = ["uniform", "large"] if kind == "f32" else ["uniform", "sine", "extreme"]
    for d_i, dist in enumerate(dists):
        x = np.stack([refs.rand_input(kind, 2 * n, seed=31 * n + 7 * d_i + r, dist=dist) for r in range(3)])
        for ifft in (0, 1, 2):          # 2: not == 1, so a forward transform
            for bitrev in (0, 1):
                a = oracle.cfft_many(kind, n, x, ifft, bitrev)
                b = ref.cfft_many(kind, n, x, ifft, bitrev)
                assert a.tobytes() == b.tobytes(), (dist, ifft, bitrev)


def test_cfft_special_values(oracle, ref):
    """zeros, signed zeros, infinities and NaNs propagate identically."""
    n = 1024
    x = np.zeros(2 * n, dtype=np.float32)
    x[::7] = -0.0
    x[5] = np.inf
    x[11] = np.nan
    for ifft in (0, 1):
        a, b = oracle.cfft("f32", n, x, ifft, 1), ref.cfft("f32", n, x, ifft, 1)
        assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("n", [32, 64, 128, 256, 512, 1024, 2048, 4096])
def test_rfft_oracle_equals_reference(oracle, ref, n):
    for seed in range(3):
        x = refs.rand_input("f32", n, seed=seed + n)
        for ifft in (0, 1):
            (a, pa), (b, pb) = oracle.rfft(n, x, ifft), ref.rfft(n, x, ifft)
            assert a.tobytes() == b.tobytes() and pa.tobytes() == pb.tobytes()


def fir_case(kind, taps, blocks, seed):
    """Coefficients and blocks for a FIR kind: f32 normal/uniform, fixed point full range."""
    rng = np.random.default_rng(seed)
    if kind == "f32":
        return (rng.standard_normal(taps).astype(np.float32),
                [rng.uniform(-1, 1, b).astype(np.float32) for b in blocks])
    bits, dt = {"q15": (15, np.int16), "q31": (31, np.int32), "q7": (7, np.int8)}[kind.split("_")[-1]]
    lo, hi = -(1 << bits), (1 << bits) - 1
    return (rng.integers(lo, hi, taps, endpoint=True).astype(dt),
            [rng.integers(lo, hi, b, endpoint=True).astype(dt) for b in blocks])


FIR_KINDS = ["f32", "q15", "q31", "fast_q15", "fast_q31", "q7"]


@pytest.mark.parametrize("kind", FIR_KINDS)
@pytest.mark.parametrize("taps,blocks", [(128, [4096, 4096]), (2, [1, 3, 5]), (29, [32] * 10), (64, [7, 100, 33]),
                                         (1, [16, 16]), (130, [2049, 3])])
def test_fir_oracle_equals_reference(oracle, ref, kind, taps, blocks):
    if kind.endswith("q15") and taps % 2:
        pytest.skip("q15: even numTaps only")
    c, xs = fir_case(kind, taps, blocks, taps)
    (ya, sa), (yb, sb) = oracle.fir(kind, c, xs), ref.fir(kind, c, xs)
    for u, v in zip(ya, yb):
        assert u.tobytes() == v.tobytes()
    assert sa.tobytes() == sb.tobytes()


def test_fir_q15_all_min_wraps_like_reference(oracle, ref):
    c = np.full(8, -32768, dtype=np.int16)
    x = [np.full(8191, -32768, dtype=np.int16)]
    (ya, _), (yb, _) = oracle.fir("q15", c, x), ref.fir("q15", c, x)
    assert ya[0].tobytes() == yb[0].tobytes()
    assert len(np.unique(ya[0])) > 1      # the grouped outputs wrap, the tail does not


@pytest.mark.parametrize("kind,word,taps", [("q31", -(1 << 31), 6), ("fast_q31", -(1 << 31), 6),
                                            ("fast_q15", -32768, 6), ("q31", (1 << 31) - 1, 6),
                                            ("fast_q31", (1 << 31) - 1, 6), ("q7", -128, 6), ("q7", -128, 1000)])
def test_fir_extreme_words_wrap_like_reference(oracle, ref, kind, word, taps):
    """All-extreme samples and taps: the q63 / q31 accumulators wrap (gcc x86-64 adds); q7 at
    1000 taps saturates (16384 * 1000 >> 7 > 127)."""
    dt = {"q15": np.int16, "q31": np.int32, "q7": np.int8}[kind.split("_")[-1]]
    c = np.full(taps, word, dtype=dt)
    x = [np.full(37, word, dtype=dt)]
    (ya, _), (yb, _) = oracle.fir(kind, c, x), ref.fir(kind, c, x)
    assert ya[0].tobytes() == yb[0].tobytes()


@pytest.mark.parametrize("m,k,n", [(1, 1, 1), (7, 13, 5), (40, 40, 40), (64, 3, 65)])
def test_mat_mult_oracle_equals_reference(oracle, ref, m, k, n):
    rng = np.random.default_rng(m + k + n)
    a = rng.uniform(-1, 1, (m, k)).astype(np.float32)
    b = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    (sa, ca), (sb, cb) = oracle.mat_mult(a, b), ref.mat_mult(a, b)
    assert sa == sb == 0 and ca.tobytes() == cb.tobytes()


def _fma_f32_exact(a, b, c):
    """round-to-nearest-even f32 of the exact a*b + c (Fractions; no double rounding)."""
    from fractions import Fraction
    s = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
    f = np.float32(float(s))
    cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
    best = min(cands, key=lambda v: (abs(Fraction(float(v)) - s), int(np.float32(v).view(np.uint32)) & 1))
    if s == 0:       # IEEE 754 RN: -0 only when a*b and c are both -0
        ab = float(a) * float(b)
        both_neg = ab == 0 and float(c) == 0 and np.signbit(ab) and np.signbit(c)
        return np.float32(-0.0) if both_neg else np.float32(0.0)
    return np.float32(best)


@pytest.mark.parametrize("m,k,n,scale", [(3, 5, 4, 1.0), (4, 17, 3, 1.0), (3, 9, 3, 2.0 ** -66), (2, 33, 2, 1e3)])
def test_mat_mult_fmaf_oracle_is_an_exact_fma_chain(oracle, ref, m, k, n, scale):
    """oracle_mat_mult_f32_fmaf (the GPU kernel's stated semantics, v_mfma_f32_32x32x2_f32)
    equals a k-ordered chain of correctly rounded fused multiply-adds computed with exact
    rationals -- including subnormal products (scale 2^-66: |a b| < 2^-126) -- and stays within
    the f32 summation bound of the reference's own mul-then-add arm_mat_mult_f32."""
    rng = np.random.default_rng(m * 100 + k)
    a = (rng.uniform(-1, 1, (m, k)) * scale).astype(np.float32)
    b = (rng.uniform(-1, 1, (k, n)) * scale).astype(np.float32)
    st, got = oracle.mat_mult_fmaf(a, b)
    assert st == 0
    want = np.zeros((m, n), dtype=np.float32)
    for i in range(m):
        for j in range(n):
            acc = np.float32(0.0)
            for kk in range(k):
                acc = _fma_f32_exact(a[i, kk], b[kk, j], acc)
            want[i, j] = acc
    assert got.tobytes() == want.tobytes()
    _, r = ref.mat_mult(a, b)
    mag = np.abs(a).astype(np.float64) @ np.abs(b).astype(np.float64)
    assert np.all(np.abs(got.astype(np.float64) - r) <= 2 * k * 2.0 ** -24 * mag + 2.0 ** -149 * k)


@pytest.mark.parametrize("kind", ["q7", "q15", "q31"])
@pytest.mark.parametrize("m,k,n,fill", [(1, 1, 1, None), (7, 13, 5, None), (33, 70, 17, None), (8, 64, 9, "min"),
                                        (8, 64, 9, "max"), (3, 65535, 2, "min"), (2, 65535, 3, None)])
def test_mat_mult_fixed_oracle_equals_reference(oracle, ref, kind, m, k, n, fill):
    """q7 (arm_mat_mult_q7.c:689-790), q15, q31: full-range, all-minimum / all-maximum inputs and
    K = 65535 (the largest uint16_t length: q7's q31 sum reaches -(2^14)*65535 without wrapping)."""
    bits, dt = {"q7": (7, np.int8), "q15": (15, np.int16), "q31": (31, np.int32)}[kind]
    rng = np.random.default_rng(m * 31 + k + n)
    if fill is None:
        a = rng.integers(-(1 << bits), 1 << bits, (m, k)).astype(dt)
        b = rng.integers(-(1 << bits), 1 << bits, (k, n)).astype(dt)
    else:
        v = -(1 << bits) if fill == "min" else (1 << bits) - 1
        a, b = np.full((m, k), v, dt), np.full((k, n), v, dt)
    (sa, ca), (sb, cb) = oracle.mat_mult_fixed(kind, a, b), ref.mat_mult_fixed(kind, a, b)
    assert sa == sb == 0 and ca.tobytes() == cb.tobytes()


@pytest.mark.parametrize("kind", ["f32", "q15", "q31", "q7"])
@pytest.mark.parametrize("la,lb", [(1, 1), (5, 3), (3, 5), (64, 64), (100, 7), (7, 100), (1000, 129), (129, 1000),
                                   (33, 1), (1, 33), (10, 37), (65, 64)])
def test_conv_oracle_equals_reference(oracle, ref, kind, la, lb):
    c, xs = fir_case(kind, lb, [la], la * 13 + lb)
    assert oracle.conv(kind, xs[0], c).tobytes() == ref.conv(kind, xs[0], c).tobytes()


@pytest.mark.parametrize("kind", ["fast_q15", "fast_q31"])
@pytest.mark.parametrize("m,k,n", [(1, 1, 1), (2, 3, 4), (5, 7, 3), (16, 16, 16), (33, 17, 9), (8, 100, 5)])
def test_mat_mult_fast_oracle_equals_reference(oracle, ref, kind, m, k, n):
    """arm_mat_mult_fast_q15 / _q31 (modular sums; odd shapes hit the reference's 2x2-block
    remainder loops), full-range and all-minimum inputs."""
    rng = np.random.default_rng(m * 100 + k * 10 + n)
    dt, bits = (np.int16, 15) if kind.endswith("q15") else (np.int32, 31)
    for fill in (None, "min"):
        if fill is None:
            a = rng.integers(-(1 << bits), 1 << bits, (m, k)).astype(dt)
            b = rng.integers(-(1 << bits), 1 << bits, (k, n)).astype(dt)
        else:
            a, b = np.full((m, k), -(1 << bits), dt), np.full((k, n), -(1 << bits), dt)
        (sa, ca), (sb, cb) = oracle.mat_mult_fixed(kind, a, b), ref.mat_mult_fixed(kind, a, b)
        assert sa == sb == 0 and ca.tobytes() == cb.tobytes(), fill
