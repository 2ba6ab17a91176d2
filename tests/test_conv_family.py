"""Convolution / correlation family: arm_correlate_{f32,q15,q31,fast_q15,fast_q31},
arm_conv_partial_{f32,q15,q31}, arm_conv_fast_{q15,q31} (+ arm_conv_* re-checked through the
same kernels).

CPU: the oracle restatement (oracle/src/oracle_conv.c) equals the reference build
(oracle/_ref) bit for bit over length pairs that hit every stage of the reference's loop
structure (srcBLen < 4, remainders mod 4, both length orders) and over input distributions
that exercise wrap-around and the fast-q15 single-sample __SMLAD term (all-negative data).
GPU: the product (drop-in and batched, both kernels: windowed and direct) equals the
reference build bit for bit.
"""
import numpy as np
import pytest

from cmsisdsp_amd import _abi

FULL = list(_abi.CONV_FULL)
PARTIAL = list(_abi.CONV_PARTIAL)
PARTIAL_FAST = list(_abi.CONV_PARTIAL_FAST)
DT = {"f32": np.float32, "q15": np.int16, "q31": np.int32, "q7": np.int8}
SMALL = [(a, b) for a in (1, 2, 3, 4, 5, 7, 8, 9, 13, 16, 17, 33) for b in (1, 2, 3, 4, 5, 6, 7, 9, 12, 13, 17, 33)]


def gen(kind, n, rng, dist):
    if kind == "f32":
        return (rng.standard_normal(n) * (1e3 if dist == "large" else 1)).astype(np.float32)
    info = np.iinfo(DT[kind])
    if dist == "full":
        return rng.integers(info.min, info.max, n, endpoint=True).astype(DT[kind])
    if dist == "neg":               # every single-sample fast-q15 MAC takes the +1 term
        return rng.integers(info.min, 0, n).astype(DT[kind])
    if dist == "min":
        return np.full(n, info.min, DT[kind])
    return rng.integers(-(2 ** (info.bits - 4)), 2 ** (info.bits - 4), n).astype(DT[kind])


def dists(kind):
    return ("small", "large") if kind == "f32" else ("small", "full", "neg", "min")


def partial_ranges(la, lb):
    L = la + lb - 1
    out = set()
    for first in {0, 1, 3, lb - 1, lb, la - 1, la, L // 2, L - 3, L - 1}:
        for num in {1, 2, 5, L - first, (L - first) // 2}:
            if 0 <= first < L and 1 <= num and first + num <= L:
                out.add((first, num))
    return sorted(out)


# ------------------------------------------------------------------ CPU: oracle == reference
@pytest.mark.parametrize("fn", FULL)
def test_conv_family_oracle_equals_reference(oracle, ref, fn):
    kind = fn.split("_")[-1]
    rng = np.random.default_rng(len(fn))
    for la, lb in SMALL + [(200, 129), (129, 200), (1000, 64)]:
        for dist in dists(kind):
            a, b = gen(kind, la, rng, dist), gen(kind, lb, rng, dist)
            (yo, _), (yr, _) = oracle.conv_family(fn, a, b, fill=7), ref.conv_family(fn, a, b, fill=7)
            assert yo.tobytes() == yr.tobytes(), (la, lb, dist)


@pytest.mark.parametrize("fn", PARTIAL)
def test_conv_partial_oracle_equals_reference(oracle, ref, fn):
    kind = fn.split("_")[-1]
    rng = np.random.default_rng(3)
    for la, lb in [(1, 1), (5, 3), (3, 5), (17, 9), (9, 17), (40, 40), (100, 7)]:
        for dist in dists(kind):
            a, b = gen(kind, la, rng, dist), gen(kind, lb, rng, dist)
            for first, num in partial_ranges(la, lb):
                (yo, so), (yr, sr) = oracle.conv_family(fn, a, b, first, num, 7), ref.conv_family(fn, a, b, first, num, 7)
                assert so == sr == 0 and yo.tobytes() == yr.tobytes(), (la, lb, dist, first, num)
            L = la + lb - 1
            for first, num in ((0, L + 1), (L, 1), (L - 1, 2)):      # out of range: ARM_MATH_ARGUMENT_ERROR
                (yo, so), (yr, sr) = oracle.conv_family(fn, a, b, first, num, 7), ref.conv_family(fn, a, b, first, num, 7)
                assert so == sr == _abi.ARM_MATH_ARGUMENT_ERROR and yo.tobytes() == yr.tobytes()


def test_fast_q15_single_sample_term_is_real(ref, oracle):
    """The reference's single-sample __SMLAD (none.h:455-463) adds +1 per MAC with both samples
    negative: (-1) * (-32767) = 32767 >> 15 = 0 exactly, but output 0 of arm_conv_fast_q15
    (one single-sample MAC) is (32767 + 1) >> 15 = 1; the stage-2 output (plain sums) is not."""
    a = np.full(5, -1, np.int16)
    b = np.full(3, -32767, np.int16)
    y, _ = ref.conv_family("conv_fast_q15", a, b)
    assert y[0] == 1 and y[2] == (3 * 32767) >> 15
    assert oracle.conv_family("conv_fast_q15", a, b)[0].tobytes() == y.tobytes()


# ------------------------------------------------------------------ GPU parity
GPU_PAIRS = [(1, 1), (5, 3), (3, 5), (7, 100), (100, 7), (4100, 129), (129, 4100), (4096, 1024), (2000, 1500),
             (1500, 2000), (33, 1), (17, 13)]


@pytest.mark.gpu
@pytest.mark.parametrize("fn", FULL)
def test_conv_family_dropin_bitexact(dsp, torch_gpu, ref, fn):
    """Drop-in calls (host buffers), both length orders, the windowed kernel (srcBLen <= 1024)
    and the direct kernel beyond it; untouched correlate words keep the caller's fill."""
    kind = fn.split("_")[-1]
    rng = np.random.default_rng(11)
    for la, lb in GPU_PAIRS:
        for dist in dists(kind)[:3]:
            a, b = gen(kind, la, rng, dist), gen(kind, lb, rng, dist)
            got, _ = dsp.arm_conv_family(fn, a, b, fill=5)
            want, _ = ref.conv_family(fn, a, b, fill=5)
            assert got.tobytes() == want.tobytes(), (la, lb, dist)


@pytest.mark.gpu
@pytest.mark.parametrize("fn", PARTIAL)
def test_conv_partial_dropin_bitexact(dsp, torch_gpu, ref, fn):
    kind = fn.split("_")[-1]
    rng = np.random.default_rng(12)
    for la, lb in [(5, 3), (3, 5), (300, 40), (40, 300), (5000, 129), (1500, 1100)]:
        a, b = gen(kind, la, rng, "full" if kind != "f32" else "small"), gen(kind, lb, rng, "small")
        for first, num in partial_ranges(la, lb):
            got, sg = dsp.arm_conv_family(fn, a, b, first, num, fill=9)
            want, sw = ref.conv_family(fn, a, b, first, num, fill=9)
            assert sg == sw == 0 and got.tobytes() == want.tobytes(), (la, lb, first, num)
        L = la + lb - 1
        got, sg = dsp.arm_conv_family(fn, a, b, L - 1, 2, fill=9)
        assert sg == _abi.ARM_MATH_ARGUMENT_ERROR and (got == 9).all()


@pytest.mark.gpu
@pytest.mark.parametrize("fn", FULL + PARTIAL)
@pytest.mark.parametrize("la,lb", [(3000, 77), (77, 3000), (2048, 1300)])
def test_conv_family_batch(dsp, torch_gpu, ref, fn, la, lb):
    """Batched device API: per-item operands and a shared pSrcB; partial outputs compact."""
    kind = fn.split("_")[-1]
    batch = 5
    rng = np.random.default_rng(la + lb)
    A = np.stack([gen(kind, la, rng, "full" if kind != "f32" else "small") for _ in range(batch)])
    B = np.stack([gen(kind, lb, rng, "neg" if kind == "q15" else "small") for _ in range(batch)])
    tdt = {"f32": torch_gpu.float32, "q15": torch_gpu.int16, "q31": torch_gpu.int32, "q7": torch_gpu.int8}[kind]
    L = la + lb - 1
    first, num = (lb // 2, L - lb) if fn in PARTIAL else (0, 0)
    width = num if fn in PARTIAL else (2 * max(la, lb) - 1 if fn.startswith("correlate") else L)
    for shared in (False, True):
        dA = torch_gpu.from_numpy(A).cuda()
        dB = torch_gpu.from_numpy(B[0].copy()).cuda() if shared else torch_gpu.from_numpy(B).cuda()
        out = torch_gpu.full((batch, width), 3, dtype=tdt, device="cuda")
        dsp.conv_family_batch(fn, dA, dB, out, first, num)
        got = out.cpu().numpy()
        for i in range(batch):
            want, _ = ref.conv_family(fn, A[i], B[0] if shared else B[i], first, num, fill=3)
            if fn in PARTIAL:
                want = want[first:first + num]
            assert got[i].tobytes() == want.tobytes(), (shared, i)


@pytest.mark.gpu
@pytest.mark.parametrize("fn", PARTIAL_FAST)
def test_conv_partial_fast(dsp, torch_gpu, ref, fn):
    """arm_conv_partial_fast_*: the words of arm_conv_fast_* over the range (the reference's
    own partial-fast bodies read outside the inputs for most ranges on the host build, so
    parity is pinned to the reference's arm_conv_fast_*), drop-in and batched."""
    kind = fn.split("_")[-1]
    full = fn.replace("partial_", "")
    rng = np.random.default_rng(13)
    for la, lb in [(5, 3), (3, 5), (300, 40), (40, 300), (5000, 129), (1500, 1100)]:
        a, b = gen(kind, la, rng, "neg"), gen(kind, lb, rng, "full")
        want, _ = ref.conv_family(full, a, b)
        for first, num in partial_ranges(la, lb):
            got, st = dsp.arm_conv_family(fn, a, b, first, num, fill=9)
            assert st == 0 and got[first:first + num].tobytes() == want[first:first + num].tobytes(), (la, lb, first, num)
            assert (got[:first] == 9).all() and (got[first + num:] == 9).all()
        assert dsp.arm_conv_family(fn, a, b, la + lb - 2, 2)[1] == _abi.ARM_MATH_ARGUMENT_ERROR
    la, lb, batch = 2500, 300, 4
    A = np.stack([gen(kind, la, rng, "full") for _ in range(batch)])
    B = gen(kind, lb, rng, "neg")
    tdt = torch_gpu.int16 if kind == "q15" else torch_gpu.int32
    first, num = 100, 2600
    out = torch_gpu.zeros((batch, num), dtype=tdt, device="cuda")
    dsp.conv_family_batch(fn, torch_gpu.from_numpy(A).cuda(), torch_gpu.from_numpy(B).cuda(), out, first, num)
    got = out.cpu().numpy()
    for i in range(batch):
        assert got[i].tobytes() == ref.conv_family(full, A[i], B)[0][first:first + num].tobytes(), i
