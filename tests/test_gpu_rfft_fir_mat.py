"""GPU parity: real FFT (fast) f32, FIR f32/q15, matrix multiply f32 vs the reference.

rfft / FIR: bit-exact against oracle/_ref.  mat_mult: MFMA f32 accumulates as an fmaf
chain (one rounding per term fewer than the reference's mul-then-add), so the bar is the
reference test's own tolerance (Testing/Source/Tests/BinaryTestsF32.cpp:5,13-17:
rel 1e-6 / abs 1e-5 at dims <= 40) plus a per-element bound at large sizes:
|C - C64|ij <= K * 2^-24 * (|A||B|)ij, 2x that against the reference build, and a bf16
negative control that must fail it.
"""
import numpy as np
import pytest

import refs

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ RFFT fast
@pytest.mark.parametrize("n", [32, 64, 128, 256, 512, 1024, 2048, 4096])
@pytest.mark.parametrize("ifft", [0, 1, 2])   # 2: merge + forward inner CFFT (unfused path)
def test_rfft_batch_bitexact(dsp, torch_gpu, ref, n, ifft):
    """out AND the side effect on p equal the reference's on every direction: the forward leaves
    the inner CFFT's output in p, the inverse (merge_rfft_f32, arm_rfft_fast_f32.c:405-462,
    684-688) never writes p.  With ARM_MI355X_RFFT_P_SCRATCH out is unchanged bit for bit and the
    inverse still leaves p alone."""
    torch = torch_gpu
    batch = 19
    x = np.stack([refs.rand_input("f32", n, seed=n + r + 100 * ifft) for r in range(batch)])
    want = np.stack([ref.rfft(n, x[r], ifft)[0] for r in range(batch)])
    want_p = np.stack([ref.rfft(n, x[r], ifft)[1] for r in range(batch)])
    if ifft:
        assert want_p.tobytes() == x.tobytes()        # the reference's inverse leaves p alone
    S = dsp.const_instance(f"arm_rfft_fast_sR_f32_len{n}")
    for p_scratch in (False, True):
        p = torch.from_numpy(x.copy()).cuda()
        out = torch.zeros_like(p)
        dsp.rfft_fast_batch(S, p, out, ifft, p_scratch=p_scratch)
        torch.cuda.synchronize()
        assert out.cpu().numpy().tobytes() == want.tobytes(), p_scratch
        if not p_scratch or ifft:
            assert p.cpu().numpy().tobytes() == want_p.tobytes(), p_scratch


def test_rfft_batch_ex_rejects_unknown_flags(dsp, torch_gpu):
    import ctypes as C
    S = dsp.const_instance("arm_rfft_fast_sR_f32_len1024")
    p = torch_gpu.zeros((2, 1024), device="cuda")
    st = dsp.lib.arm_rfft_fast_f32_batch_ex(C.byref(S), C.c_void_p(p.data_ptr()), C.c_void_p(p.data_ptr()), 2, 0, 2,
                                            None)
    assert st == dsp.ARM_MATH_ARGUMENT_ERROR


@pytest.mark.parametrize("n", [32, 1024, 4096])
def test_rfft_dropin(dsp, torch_gpu, ref, n):
    """The drop-in on host buffers: pOut and p after the call equal the reference's, both ways
    (forward: p holds the inner CFFT output; inverse: p untouched)."""
    import ctypes as C
    x = refs.rand_input("f32", n, seed=n)
    for ifft in (0, 1):
        S = dsp.arm_rfft_fast_instance_f32()
        assert dsp.arm_rfft_fast_init_f32(S, n) == 0
        assert dsp.arm_rfft_fast_f32(S, x, ifft).tobytes() == ref.rfft(n, x, ifft)[0].tobytes()
        p = x.copy()
        out = np.zeros(n, dtype=np.float32)
        dsp.lib.arm_rfft_fast_f32(C.byref(S), p.ctypes.data, out.ctypes.data, ifft)
        want, want_p = ref.rfft(n, x, ifft)
        assert out.tobytes() == want.tobytes() and p.tobytes() == want_p.tobytes(), ifft


# ------------------------------------------------------------------ FIR
def _fir_batched(dsp, torch, kind, coeffs, blocks_per_filter):
    """blocks_per_filter: [batch][calls] arrays; runs the batched API call by call."""
    import ctypes as C
    base = "f32" if kind == "f32_fma" else kind.split("_")[-1]
    dt = {"f32": np.float32, "q15": np.int16, "q31": np.int32, "q7": np.int8}[base]
    batch, calls = len(blocks_per_filter), len(blocks_per_filter[0])
    c = np.ascontiguousarray(coeffs, dtype=dt)
    S = {"f32": dsp.arm_fir_instance_f32, "q15": dsp.arm_fir_instance_q15, "q31": dsp.arm_fir_instance_q31,
         "q7": dsp.arm_fir_instance_q7}[base]()
    S.numTaps = len(c)
    dc = torch.from_numpy(c.copy()).cuda()
    S.pCoeffs = C.cast(dc.data_ptr(), S._fields_[2][1])
    hist = torch.zeros((batch, max(len(c) - 1, 0)), dtype=dc.dtype, device="cuda")
    outs = []
    for k in range(calls):
        src = torch.from_numpy(np.stack([blocks_per_filter[f][k] for f in range(batch)]).astype(dt)).cuda()
        dst = torch.empty_like(src)
        dsp.fir_batch(S, src, dst, hist, kind=kind)
        outs.append(dst.cpu().numpy())
    torch.cuda.synchronize()
    return outs, hist.cpu().numpy()


FIR_KINDS = ["f32", "q15", "q31", "fast_q15", "fast_q31", "q7"]


@pytest.mark.parametrize("kind", FIR_KINDS)
@pytest.mark.parametrize("taps,block", [(128, 4096), (29, 32), (2, 7), (64, 100), (130, 2049), (1, 64),
                                        (6, 50), (240, 1000), (242, 777), (256, 4100), (1024, 3000), (518, 2048)])
def test_fir_batch_bitexact_two_calls(dsp, torch_gpu, ref, kind, taps, block):
    """Each filter runs two consecutive blocks: the state carry must make them equal one
    long call (FIRF32.cpp:116-124 does the same two-call split)."""
    if kind.endswith("q15") and taps % 2:
        pytest.skip("q15 FIR requires an even numTaps (arm_fir_init_q15.c:95-106)")
    rng = np.random.default_rng(taps * 7 + block)
    batch = 5
    if kind == "f32":
        coeffs = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
        blocks = [[rng.uniform(-1, 1, block).astype(np.float32) for _ in range(2)] for _ in range(batch)]
    else:
        bits, dt = {"q15": (15, np.int16), "q31": (31, np.int32), "q7": (7, np.int8)}[kind.split("_")[-1]]
        lo, hi = -(1 << bits), (1 << bits) - 1
        coeffs = rng.integers(lo, hi, taps, endpoint=True).astype(dt)
        blocks = [[rng.integers(lo, hi, block, endpoint=True).astype(dt) for _ in range(2)]
                  for _ in range(batch)]
    got, hist = _fir_batched(dsp, torch_gpu, kind, coeffs, blocks)
    for f in range(batch):
        want, state = ref.fir(kind, coeffs, blocks[f])
        for k in range(2):
            assert got[k][f].tobytes() == want[k].tobytes(), (f, k)
        assert hist[f].tobytes() == state[:taps - 1].tobytes()


@pytest.mark.parametrize("taps,block,fill", [(128, 4096, None), (2, 4096, None), (8, 1000, "min"), (64, 4100, "mixed"),
                                             (130, 2049, None), (158, 4096, "max"), (160, 8195, None),
                                             (128, 4096, "min"), (16, 4096, "wrap")])
@pytest.mark.parametrize("kind", ["q15", "fast_q15"])
def test_fir_q15_mfma_path(dsp, torch_gpu, ref, taps, block, fill, kind):
    """arm_fir_q15 through the i8-MFMA kernel (fir_mfma.hip: even numTaps <= 160 and >= 256
    (filter, 4096-output chunk) items per call): 260 filters, two calls each (state carry), every
    word of 12 filters against the reference build -- random full range, all -32768 / 32767 (the
    plane sums at their extremes, the output saturating), mixed extremes, and taps holding a
    (-32768, -32768) pair over all -32768 input (the __SMLALD pair wrap: the kernel's exact pair-wise
    path).  arm_fir_fast_q15 runs the same kernel with the modular (q31_t wrap) epilogue."""
    rng = np.random.default_rng(taps * 31 + block)
    batch = 260
    if fill == "min" or fill == "wrap":
        coeffs = rng.integers(-32768, 32767, taps, endpoint=True).astype(np.int16)
        if fill == "wrap":
            coeffs[4:6] = -32768
        mk = lambda: np.full(block, -32768, np.int16)
    elif fill == "max":
        coeffs = np.full(taps, 32767, np.int16)
        mk = lambda: np.full(block, 32767, np.int16)
    elif fill == "mixed":
        vals = np.array([-32768, 32767, 0, -1, 1], np.int16)
        coeffs = rng.choice(vals, taps)
        mk = lambda: rng.choice(vals, block)
    else:
        coeffs = rng.integers(-32768, 32767, taps, endpoint=True).astype(np.int16)
        mk = lambda: rng.integers(-32768, 32767, block, endpoint=True).astype(np.int16)
    blocks = [[mk() for _ in range(2)] for _ in range(batch)]
    got, hist = _fir_batched(dsp, torch_gpu, kind, coeffs, blocks)
    for f in (0, 1, 7, 63, 64, 100, 128, 129, 200, 255, 258, 259):
        want, state = ref.fir(kind, coeffs, blocks[f])
        for k in range(2):
            assert got[k][f].tobytes() == want[k].tobytes(), (f, k, np.argwhere(got[k][f] != want[k])[:4])
        assert hist[f].tobytes() == state[:taps - 1].tobytes()


@pytest.mark.parametrize("taps,block,fill", [(128, 4096, None), (1, 4096, None), (161, 4096, None), (64, 4100, "mixed"),
                                             (130, 2049, None), (127, 4096, "big1"), (31, 4096, "big4"),
                                             (64, 4096, "big7"), (128, 4096, "min"), (128, 4096, "max"),
                                             (160, 8195, None), (33, 1000, "big2")])
def test_fir_q31_mfma_path(dsp, torch_gpu, ref, taps, block, fill):
    """arm_fir_q31 through the i8-MFMA kernel (fir_mfma.hip: numTaps <= 161 and >= 256 (filter,
    4096-output chunk) items per call): 260 filters, two calls each (state carry), every word of 12
    filters against the reference build -- random full range, all INT_MIN / INT_MAX (the class sums
    at their extremes, the q63 sum wrapping), mixed extremes, and taps above 0x7F7F7F7F (no
    balanced 4-digit form: 1, 2 and 4 of them corrected per output, 7 taking the exact
    per-output path)."""
    rng = np.random.default_rng(taps * 37 + block)
    batch = 260
    lo, hi = -(1 << 31), (1 << 31) - 1
    coeffs = rng.integers(lo, hi, taps, endpoint=True).astype(np.int32)
    mk = lambda: rng.integers(lo, hi, block, endpoint=True).astype(np.int32)
    if fill == "min":
        mk = lambda: np.full(block, lo, np.int32)
    elif fill == "max":
        coeffs = np.full(taps, hi, np.int32)
        mk = lambda: np.full(block, hi, np.int32)
    elif fill == "mixed":
        vals = np.array([lo, hi, 0, -1, 1, 0x7F7F7F7F, 0x7F7F7F80], np.int32)
        coeffs = rng.choice(vals, taps)
        mk = lambda: rng.choice(vals, block)
    elif fill and fill.startswith("big"):
        coeffs = np.clip(coeffs, lo, 0x7F7F7F7F).astype(np.int32)
        idx = rng.choice(taps, int(fill[3:]), replace=False)
        coeffs[idx] = rng.integers(0x7F7F7F80, hi, len(idx), endpoint=True)
    blocks = [[mk() for _ in range(2)] for _ in range(batch)]
    got, hist = _fir_batched(dsp, torch_gpu, "q31", coeffs, blocks)
    for f in (0, 1, 7, 63, 64, 100, 128, 129, 200, 255, 258, 259):
        want, state = ref.fir("q31", coeffs, blocks[f])
        for k in range(2):
            assert got[k][f].tobytes() == want[k].tobytes(), (f, k, np.argwhere(got[k][f] != want[k])[:4])
        assert hist[f].tobytes() == state[:taps - 1].tobytes()


@pytest.mark.parametrize("taps,block,fill", [(128, 4096, None), (1, 4096, None), (157, 4096, None), (64, 4100, "mixed"),
                                             (130, 2049, None), (33, 1001, None), (128, 4096, "min"),
                                             (128, 4096, "max"), (100, 8195, None)])
def test_fir_q7_mfma_path(dsp, torch_gpu, ref, taps, block, fill):
    """arm_fir_q7 through the i8-MFMA kernel (fir_mfma.hip: numTaps <= 157 and >= 256 (filter,
    4096-output chunk) items per call; ragged blocks give every filter its own window shift d):
    260 filters, two calls each (state carry), every word of 12 filters against the reference
    build -- random full range, all -128 / 127 (the output saturating both ways), mixed extremes."""
    rng = np.random.default_rng(taps * 41 + block)
    batch = 260
    coeffs = rng.integers(-128, 127, taps, endpoint=True).astype(np.int8)
    mk = lambda: rng.integers(-128, 127, block, endpoint=True).astype(np.int8)
    if fill == "min":
        coeffs = np.full(taps, -128, np.int8)
        mk = lambda: np.full(block, -128, np.int8)
    elif fill == "max":
        coeffs = np.full(taps, 127, np.int8)
        mk = lambda: np.full(block, -128, np.int8)
    elif fill == "mixed":
        vals = np.array([-128, 127, 0, -1, 1], np.int8)
        coeffs = rng.choice(vals, taps)
        mk = lambda: rng.choice(vals, block)
    blocks = [[mk() for _ in range(2)] for _ in range(batch)]
    got, hist = _fir_batched(dsp, torch_gpu, "q7", coeffs, blocks)
    for f in (0, 1, 7, 63, 64, 100, 128, 129, 200, 255, 258, 259):
        want, state = ref.fir("q7", coeffs, blocks[f])
        for k in range(2):
            assert got[k][f].tobytes() == want[k].tobytes(), (f, k, np.argwhere(got[k][f] != want[k])[:4])
        assert hist[f].tobytes() == state[:taps - 1].tobytes()


def test_fir_q15_pairwrap_extreme(dsp, torch_gpu, ref):
    """All -32768 input and taps: the __SMLALD pair sum wraps in int32 on the unrolled
    outputs but not on the blockSize%4 tail (arm_fir_q15.c:482-640 vs :649-681)."""
    taps, block = 8, 4099
    coeffs = np.full(taps, -32768, dtype=np.int16)
    blocks = [[np.full(block, -32768, dtype=np.int16)]]
    got, _ = _fir_batched(dsp, torch_gpu, "q15", coeffs, blocks)
    want, _ = ref.fir("q15", coeffs, blocks[0])
    assert got[0][0].tobytes() == want[0].tobytes()


@pytest.mark.parametrize("taps", [8, 240, 256, 1024])
@pytest.mark.parametrize("pattern", ["neg", "alt"])
def test_fir_q15_extremes_split_path(dsp, torch_gpu, ref, taps, pattern):
    """Largest magnitudes the split (256*H + L) accumulation sees without a wrapping tap
    pair: -32768 samples against (-32768, 32767) / (-32768, -32767) coefficient pairs, across
    the int32 flush boundary (120 tap pairs) and the blockSize%4 tail."""
    block = 4099
    c = np.empty(taps, dtype=np.int16)
    c[0::2] = -32768
    c[1::2] = 32767 if pattern == "alt" else -32767
    x = np.full(block, -32768, dtype=np.int16)
    if pattern == "alt":
        x[1::2] = 32767
    got, _ = _fir_batched(dsp, torch_gpu, "q15", c, [[x]])
    want, _ = ref.fir("q15", c, [x])
    assert got[0][0].tobytes() == want[0].tobytes()


@pytest.mark.parametrize("taps", [6, 300])
def test_fir_q15_wrapping_pair_random(dsp, torch_gpu, ref, taps):
    """One (-32768, -32768) coefficient pair selects the exact int64 path; random data with
    runs of -32768 makes some pair sums wrap (unrolled outputs) and not wrap (tail)."""
    rng = np.random.default_rng(taps)
    block = 1023
    c = rng.integers(-32768, 32767, taps, endpoint=True).astype(np.int16)
    c[2:4] = -32768
    x = rng.integers(-32768, 32767, block, endpoint=True).astype(np.int16)
    x[rng.random(block) < 0.5] = -32768
    got, _ = _fir_batched(dsp, torch_gpu, "q15", c, [[x]])
    want, _ = ref.fir("q15", c, [x])
    assert got[0][0].tobytes() == want[0].tobytes()


@pytest.mark.parametrize("kind,word", [("q31", -(1 << 31)), ("fast_q31", -(1 << 31)), ("fast_q15", -32768),
                                       ("q31", (1 << 31) - 1), ("fast_q31", (1 << 31) - 1)])
def test_fir_extreme_words(dsp, torch_gpu, ref, kind, word):
    """All-extreme samples and taps: the q63 / q31 accumulators wrap exactly as the
    reference build's do."""
    dt = np.int16 if kind.endswith("q15") else np.int32
    coeffs = np.full(6, word, dtype=dt)
    blocks = [[np.full(4099, word, dtype=dt)]]
    got, _ = _fir_batched(dsp, torch_gpu, kind, coeffs, blocks)
    want, _ = ref.fir(kind, coeffs, blocks[0])
    assert got[0][0].tobytes() == want[0].tobytes()


@pytest.mark.parametrize("kind", ["q31", "fast_q31", "fast_q15"])
def test_fir_dropin_state_fixed_variants(dsp, torch_gpu, ref, kind):
    rng = np.random.default_rng(11)
    taps, block = 32, 256
    bits, dt = (15, np.int16) if kind.endswith("q15") else (31, np.int32)
    coeffs = rng.integers(-(1 << bits), (1 << bits) - 1, taps).astype(dt)
    blocks = [rng.integers(-(1 << bits), (1 << bits) - 1, block).astype(dt) for _ in range(3)]
    f = dsp.FirFastQ15(coeffs, block) if kind == "fast_q15" else dsp.FirQ31(coeffs, block, fast=kind == "fast_q31")
    want, state = ref.fir(kind, coeffs, blocks)
    for b, w in zip(blocks, want):
        assert f(b).tobytes() == w.tobytes()
    assert f.state.tobytes() == state.tobytes()


@pytest.mark.parametrize("kind", ["f32", "q15"])
def test_fir_dropin_state(dsp, torch_gpu, ref, kind):
    rng = np.random.default_rng(4)
    taps, block = 32, 256
    if kind == "f32":
        coeffs = rng.standard_normal(taps).astype(np.float32)
        blocks = [rng.uniform(-1, 1, block).astype(np.float32) for _ in range(3)]
        f = dsp.FirF32(coeffs, block)
    else:
        coeffs = rng.integers(-20000, 20000, taps).astype(np.int16)
        blocks = [rng.integers(-32768, 32767, block).astype(np.int16) for _ in range(3)]
        f = dsp.FirQ15(coeffs, block)
    want, state = ref.fir(kind, coeffs, blocks)
    for b, w in zip(blocks, want):
        assert f(b).tobytes() == w.tobytes()
    assert f.state.tobytes() == state.tobytes()   # history head AND the block copy in the tail


# ------------------------------------------------------------------ mat mult
@pytest.mark.parametrize("m,k,n", [(1, 1, 1), (4, 4, 4), (17, 33, 9), (40, 40, 40), (2, 129, 3)])
def test_mat_mult_small_reference_tolerance(dsp, torch_gpu, ref, m, k, n):
    rng = np.random.default_rng(m * 1000 + k * 10 + n)
    a = rng.uniform(-1, 1, (m, k)).astype(np.float32)
    b = rng.uniform(-1, 1, (k, n)).astype(np.float32)
    st, got = dsp.arm_mat_mult_f32(a, b)
    st_r, want = ref.mat_mult(a, b)
    assert st == 0 and st_r == 0
    np.testing.assert_allclose(got, want, rtol=1e-6, atol=1e-5)


def test_mat_mult_size_mismatch(dsp, torch_gpu):
    import ctypes as C
    A, B, Cm = dsp.arm_matrix_instance_f32(), dsp.arm_matrix_instance_f32(), dsp.arm_matrix_instance_f32()
    buf = np.zeros(64, dtype=np.float32)
    dsp.lib.arm_mat_init_f32(C.byref(A), 2, 3, buf.ctypes.data)
    dsp.lib.arm_mat_init_f32(C.byref(B), 4, 2, buf.ctypes.data)
    dsp.lib.arm_mat_init_f32(C.byref(Cm), 2, 2, buf.ctypes.data)
    assert dsp.lib.arm_mat_mult_f32(C.byref(A), C.byref(B), C.byref(Cm)) == dsp.ARM_MATH_SIZE_MISMATCH


def _elementwise_bound(a, b):
    """|C - C64|ij <= K 2^-24 (|A||B|)ij: the recursive-summation bound of an f32 dot
    product of length K (Higham, gamma_K), which the reference's own sequential sum
    (arm_mat_mult_f32.c:635-722) and an fmaf chain both satisfy."""
    k = a.shape[-1]
    return k * 2.0 ** -24 * np.einsum("...mk,...kn->...mn", np.abs(a).astype(np.float64), np.abs(b).astype(np.float64))


def _bf16(x):
    import torch
    return torch.from_numpy(x).bfloat16().double().numpy()


def _tf32(x):
    """Round f32 to a 10-bit mantissa (TF32 / xf32 operands), nearest-even."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0xFFF + ((u >> 13) & 1)) & ~np.uint64(0x1FFF)
    return u.astype(np.uint32).view(np.float32)


def _rms_ok(got, exact, mag, k):
    """Statistical f32 check: rms(|C - C64| / (|A||B|)) <= sqrt(K) 2^-24.  f32 summation (the
    reference's mul-then-add and an fmaf chain alike) sits at 0.01-0.1 of it; TF32-rounded
    operands at 5-400x (numpy simulation at K = 16 ... 1024), bf16 far above."""
    r = np.abs(got - exact) / np.maximum(mag, 1e-300)
    return float(np.sqrt(np.mean(r ** 2)) / (np.sqrt(k) * 2.0 ** -24))


def _mat_inputs(rng, shape_a, shape_b, dist):
    if dist == "uniform":
        return rng.uniform(-1, 1, shape_a).astype(np.float32), rng.uniform(-1, 1, shape_b).astype(np.float32)
    if dist == "subnormal":     # |a b| in [2^-134, 2^-132): every product subnormal, none zero
        f = lambda sh: (rng.uniform(0.5, 1.0, sh) * rng.choice([-1.0, 1.0], sh) * 2.0 ** -66).astype(np.float32)
        return f(shape_a), f(shape_b)
    if dist == "mixed":         # exponents over 2^-20 .. 2^20, exact zeros and negative zeros
        def f(sh):
            v = rng.uniform(0.5, 1.0, sh) * rng.choice([-1.0, 1.0], sh) * 2.0 ** rng.integers(-20, 21, sh)
            z = rng.uniform(0, 1, sh)
            v[z < 0.1] = 0.0
            v[(z >= 0.1) & (z < 0.2)] = -0.0
            return v.astype(np.float32)
        return f(shape_a), f(shape_b)
    raise ValueError(dist)


@pytest.mark.parametrize("m,k,n,batch,dist", [
    (1, 1, 1, 1, "uniform"), (17, 33, 9, 1, "uniform"), (300, 130, 200, 2, "uniform"),
    (64, 37, 96, 1, "uniform"), (128, 1000, 128, 1, "uniform"),          # K not a multiple of 16
    (256, 256, 256, 2, "uniform"), (128, 16, 384, 2, "uniform"),         # whole tiles: the fast kernel
    (384, 48, 128, 1, "subnormal"), (300, 130, 200, 1, "subnormal"),
    (256, 64, 128, 1, "mixed"), (65, 77, 33, 1, "mixed")])
def test_mat_mult_f32_fmaf_chain_bitexact(dsp, torch_gpu, oracle, m, k, n, batch, dist):
    """The kernel's stated semantics pinned bit for bit: C = the k-ordered fmaf chain from +0.0f
    (oracle_mat_mult_f32_fmaf; v_mfma_f32_32x32x2_f32, mat_mult_f32.hip:1-12), on both kernels,
    with subnormal products and signed zeros.  Negative control: the same chain on TF32-rounded
    operands differs from the kernel's words."""
    torch = torch_gpu
    rng = np.random.default_rng(m * 7 + k * 3 + n + len(dist))
    a, b = _mat_inputs(rng, (batch, m, k), (batch, k, n), dist)
    dc = torch.empty((batch, m, n), dtype=torch.float32, device="cuda")
    dsp.mat_mult_batch(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda(), dc)
    got = dc.cpu().numpy()
    for i in range(batch):
        st, want = oracle.mat_mult_fmaf(a[i], b[i])
        assert st == 0
        assert got[i].tobytes() == want.tobytes(), f"item {i}: {np.sum(got[i].view(np.uint32) != want.view(np.uint32))} words differ"
    if k >= 16 and dist != "subnormal":
        _, tf = oracle.mat_mult_fmaf(_tf32(a[0]), _tf32(b[0]))
        assert np.mean(tf.view(np.uint32) != got[0].view(np.uint32)) > 0.5


def test_mat_mult_f32_dropin_fmaf_bitexact(dsp, torch_gpu, oracle):
    """The host-pointer drop-in arm_mat_mult_f32 returns the same fmaf-chain words."""
    rng = np.random.default_rng(99)
    a, b = _mat_inputs(rng, (17, 33), (33, 9), "uniform")
    st, got = dsp.arm_mat_mult_f32(a, b)
    assert st == 0 and got.tobytes() == oracle.mat_mult_fmaf(a, b)[1].tobytes()


@pytest.mark.parametrize("m,k,n,batch", [(256, 256, 256, 3), (300, 130, 200, 2), (1024, 1024, 1024, 1),
                                          (128, 16, 384, 2), (384, 48, 128, 1), (128, 1000, 128, 1)])
def test_mat_mult_batch_elementwise(dsp, torch_gpu, ref, m, k, n, batch):
    """Per-element f32 bound against float64 over every item, and a negative control: the
    product of bf16-rounded operands must violate the same bound (so the check tells f32
    from bf16/tf32 inputs)."""
    torch = torch_gpu
    rng = np.random.default_rng(m + k + n)
    a = rng.uniform(-1, 1, (batch, m, k)).astype(np.float32)
    b = rng.uniform(-1, 1, (batch, k, n)).astype(np.float32)
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    dc = torch.empty((batch, m, n), dtype=torch.float32, device="cuda")
    dsp.mat_mult_batch(da, db, dc)
    got = dc.cpu().numpy().astype(np.float64)
    exact = np.einsum("bmk,bkn->bmn", a.astype(np.float64), b.astype(np.float64))
    bound = _elementwise_bound(a, b)
    assert np.all(np.abs(got - exact) <= bound)
    mag = bound / (k * 2.0 ** -24)
    assert _rms_ok(got, exact, mag, k) <= 1.0
    bf = np.einsum("bmk,bkn->bmn", _bf16(a), _bf16(b))     # negative control
    assert np.mean(np.abs(bf - exact) > bound) > 0.1
    tf = np.einsum("bmk,bkn->bmn", _tf32(a).astype(np.float64), _tf32(b).astype(np.float64))
    assert _rms_ok(tf, exact, mag, k) > 2.0                 # TF32-class operands are rejected
    if m * k * n <= 256 ** 3:   # the reference itself on one item (seconds on the host)
        st, want = ref.mat_mult(a[0], b[0])
        assert np.all(np.abs(got[0] - want) <= 2 * bound[0])


def test_mat_mult_1024_vs_reference_slice(dsp, torch_gpu, ref, oracle):
    """BASELINE configs[4] shape (1024^3): a 16-row slice of A times all of B through the
    reference's own arm_mat_mult_f32 (full K), held per element to 2 K 2^-24 (|A||B|)ij;
    the whole product per element to K 2^-24 (|A||B|)ij vs float64; and the bf16 negative
    control rejected."""
    torch = torch_gpu
    rng = np.random.default_rng(1024)
    a = rng.uniform(-1, 1, (1024, 1024)).astype(np.float32)
    b = rng.uniform(-1, 1, (1024, 1024)).astype(np.float32)
    dc = torch.empty((1, 1024, 1024), dtype=torch.float32, device="cuda")
    dsp.mat_mult_batch(torch.from_numpy(a).cuda()[None], torch.from_numpy(b).cuda()[None], dc)
    got = dc[0].cpu().numpy().astype(np.float64)
    at, bt = torch.from_numpy(a).double(), torch.from_numpy(b).double()
    exact = (at @ bt).numpy()
    bound = 1024 * 2.0 ** -24 * (at.abs() @ bt.abs()).numpy()
    assert np.all(np.abs(got - exact) <= bound)
    st, want = ref.mat_mult(a[:16], b)
    assert st == 0
    assert np.all(np.abs(got[:16] - want) <= 2 * bound[:16])
    mag = bound / (1024 * 2.0 ** -24)
    assert _rms_ok(got, exact, mag, 1024) <= 1.0
    bf = (torch.from_numpy(_bf16(a)) @ torch.from_numpy(_bf16(b))).numpy()
    assert np.mean(np.abs(bf - exact) > bound) > 0.1
    tf = (torch.from_numpy(_tf32(a)).double() @ torch.from_numpy(_tf32(b)).double()).numpy()
    assert _rms_ok(tf, exact, mag, 1024) > 2.0
    st, fm = oracle.mat_mult_fmaf(a[:16], b)              # the stated semantics, bit for bit
    assert st == 0 and dc[0, :16].cpu().numpy().tobytes() == fm.tobytes()


# ------------------------------------------------------------------ mat mult q15 / q31
@pytest.mark.parametrize("kind", ["q15", "q31", "fast_q15", "fast_q31"])
@pytest.mark.parametrize("m,k,n,fill", [(1, 1, 1, None), (5, 7, 3, None), (64, 64, 64, None), (65, 130, 67, None),
                                        (128, 2000, 96, None), (40, 64, 40, "min"), (40, 64, 40, "max"),
                                        (33, 100, 31, "mixed"), (3, 33000, 2, None),
                                        # whole 128 x 128 / 128 x 64 tiles, K % 64 == 0: the unguarded kernel
                                        (128, 128, 128, None), (256, 192, 256, "min"), (128, 320, 128, "mixed"),
                                        (256, 64, 128, "max"),
                                        # the int32 class accumulators at their exact limit (K = 32704,
                                        # every plane byte -128), and K just past a 64-deep step
                                        (2, 32704, 3, "min"), (130, 65, 129, "min")])
def test_mat_mult_fixed_bitexact(dsp, torch_gpu, ref, kind, m, k, n, fill):
    """Byte-sliced i8-MFMA kernel (K <= 32704) and the VALU kernel beyond, vs the reference
    build bit for bit, including all-extreme operands (q63 wrap for q31, saturation for q15);
    fast_q15 on the same kernels with the modular epilogue, fast_q31 on its VALU kernel."""
    bits, dt = (15, np.int16) if kind.endswith("q15") else (31, np.int32)
    rng = np.random.default_rng(m + 7 * k + 13 * n)
    lo, hi = -(1 << bits), (1 << bits) - 1
    if fill is None:
        a = rng.integers(lo, hi, (m, k), endpoint=True).astype(dt)
        b = rng.integers(lo, hi, (k, n), endpoint=True).astype(dt)
    elif fill == "mixed":
        a = rng.choice(np.array([lo, hi, 0, -1, 1], dtype=np.int64), (m, k)).astype(dt)
        b = rng.choice(np.array([lo, hi, 0, -1, 1], dtype=np.int64), (k, n)).astype(dt)
    else:
        v = lo if fill == "min" else hi
        a, b = np.full((m, k), v, dt), np.full((k, n), v, dt)
    st, got = dsp.arm_mat_mult_fixed(kind, a, b)
    st_r, want = ref.mat_mult_fixed(kind, a, b)
    assert st == 0 and st_r == 0
    assert got.tobytes() == want.tobytes(), np.argwhere(got != want)[:5]


@pytest.mark.parametrize("kind", ["q15", "q31", "fast_q15", "fast_q31"])
def test_mat_mult_fixed_batch(dsp, torch_gpu, ref, kind):
    bits, dt = (15, np.int16) if kind.endswith("q15") else (31, np.int32)
    tdt = torch_gpu.int16 if kind.endswith("q15") else torch_gpu.int32
    rng = np.random.default_rng(9)
    for (m, k, n) in ((96, 200, 80), (128, 256, 128)):        # guarded and unguarded kernels
        a = rng.integers(-(1 << bits), 1 << bits, (3, m, k)).astype(dt)
        b = rng.integers(-(1 << bits), 1 << bits, (3, k, n)).astype(dt)
        A, B = torch_gpu.from_numpy(a).cuda(), torch_gpu.from_numpy(b).cuda()
        Cm = torch_gpu.empty((3, m, n), dtype=tdt, device="cuda")
        dsp.mat_mult_batch(A, B, Cm, fast=kind.startswith("fast"))
        got = Cm.cpu().numpy()
        for i in range(3):
            assert got[i].tobytes() == ref.mat_mult_fixed(kind, a[i], b[i])[1].tobytes(), (m, i)


@pytest.mark.parametrize("kind", ["q15", "fast_q15", "q31"])
def test_mat_mult_fixed_many_tiles(dsp, torch_gpu, ref, kind):
    """Many whole tiles per launch (grid = tiles x batch = 600 workgroups): every matrix of the
    batch bit-exact against exact int64 products (checked against the reference build on a few)."""
    bits, dt = (15, np.int16) if kind.endswith("q15") else (31, np.int32)
    tdt = torch_gpu.int16 if kind.endswith("q15") else torch_gpu.int32
    rng = np.random.default_rng(21)
    batch, m, k, n = 600, 128, 128, 128
    a = rng.integers(-(1 << bits), 1 << bits, (batch, m, k)).astype(dt)
    b = rng.integers(-(1 << bits), 1 << bits, (batch, k, n)).astype(dt)
    A, B = torch_gpu.from_numpy(a).cuda(), torch_gpu.from_numpy(b).cuda()
    Cm = torch_gpu.empty((batch, m, n), dtype=tdt, device="cuda")
    dsp.mat_mult_batch(A, B, Cm, fast=kind.startswith("fast"))
    got = Cm.cpu().numpy()
    for i in (0, 1, 255, 256, 257, 511, 599):
        assert got[i].tobytes() == ref.mat_mult_fixed(kind, a[i], b[i])[1].tobytes(), i
    s = np.matmul(a.astype(np.int64), b.astype(np.int64))        # wraps mod 2^64 like the q63 sum
    if kind == "q15":
        want = np.clip(s >> 15, -32768, 32767).astype(np.int16)
    elif kind == "fast_q15":
        want = ((s.astype(np.uint64).astype(np.uint32).view(np.int32)) >> 15).astype(np.int16)
    else:
        want = (s >> 31).astype(np.int32)
    assert got.tobytes() == want.tobytes(), np.argwhere(got != want)[:5]


# ------------------------------------------------------------------ convolution
def _conv_case(kind, la, lb, seed, fill=None):
    rng = np.random.default_rng(seed)
    if kind == "f32":
        return rng.standard_normal(la).astype(np.float32), rng.standard_normal(lb).astype(np.float32)
    bits, dt = (15, np.int16) if kind == "q15" else (31, np.int32)
    if fill is not None:
        v = -(1 << bits) if fill == "min" else (1 << bits) - 1
        return np.full(la, v, dt), np.full(lb, v, dt)
    return (rng.integers(-(1 << bits), 1 << bits, la).astype(dt), rng.integers(-(1 << bits), 1 << bits, lb).astype(dt))


@pytest.mark.parametrize("kind", ["f32", "q15", "q31"])
@pytest.mark.parametrize("la,lb", [(1, 1), (5, 3), (3, 5), (100, 7), (7, 100), (5000, 129), (129, 5000), (4096, 1024),
                                   (2000, 1500), (33, 1)])
def test_conv_dropin_bitexact(dsp, torch_gpu, ref, kind, la, lb):
    """Both length orders (the reference sums in ascending index of pSrcA either way), the
    LDS path (srcBLen <= 1024) and the direct path beyond."""
    a, b = _conv_case(kind, la, lb, la * 7 + lb)
    assert dsp.arm_conv(kind, a, b).tobytes() == ref.conv(kind, a, b).tobytes()


@pytest.mark.parametrize("kind,fill", [("q15", "min"), ("q15", "max"), ("q31", "min"), ("q31", "max")])
def test_conv_extremes(dsp, torch_gpu, ref, kind, fill):
    a, b = _conv_case(kind, 300, 40, 1, fill)
    assert dsp.arm_conv(kind, a, b).tobytes() == ref.conv(kind, a, b).tobytes()


@pytest.mark.parametrize("kind", ["f32", "q15", "q31"])
@pytest.mark.parametrize("shared", [False, True])
def test_conv_batch(dsp, torch_gpu, ref, kind, shared):
    batch, la, lb = 6, 3000, 77
    A = np.stack([_conv_case(kind, la, lb, 50 + i)[0] for i in range(batch)])
    B = np.stack([_conv_case(kind, la, lb, 90 + i)[1] for i in range(batch)])
    tdt = {"f32": torch_gpu.float32, "q15": torch_gpu.int16, "q31": torch_gpu.int32}[kind]
    dA = torch_gpu.from_numpy(A).cuda()
    dB = torch_gpu.from_numpy(B[0].copy()).cuda() if shared else torch_gpu.from_numpy(B).cuda()
    out = torch_gpu.empty((batch, la + lb - 1), dtype=tdt, device="cuda")
    dsp.conv_batch(dA, dB, out)
    got = out.cpu().numpy()
    for i in range(batch):
        assert got[i].tobytes() == ref.conv(kind, A[i], B[0] if shared else B[i]).tobytes(), i


# ------------------------------------------------------------------ mat mult q7 (one i8 plane)
def _q7_operands(rng, m, k, n, fill):
    if fill is None:
        return (rng.integers(-128, 127, (m, k), endpoint=True).astype(np.int8),
                rng.integers(-128, 127, (k, n), endpoint=True).astype(np.int8))
    if fill == "mixed":
        vals = np.array([-128, 127, 0, -1, 1], dtype=np.int8)
        return rng.choice(vals, (m, k)), rng.choice(vals, (k, n))
    v = -128 if fill == "min" else 127
    return np.full((m, k), v, np.int8), np.full((k, n), v, np.int8)


def _q7_exact(a, b):
    s = np.matmul(a.astype(np.int64), b.astype(np.int64))
    return np.clip(s >> 7, -128, 127).astype(np.int8)


@pytest.mark.parametrize("m,k,n,fill", [(1, 1, 1, None), (2, 3, 2, None), (5, 7, 3, None), (64, 64, 64, None),
                                        (65, 130, 67, None), (33, 100, 31, "mixed"), (40, 64, 40, "min"),
                                        (40, 64, 40, "max"), (300, 200, 270, None), (3, 65535, 2, "min"),
                                        (17, 65535, 19, None), (130, 65, 129, "min"),
                                        # whole 256 x 256 tiles, K % 64 == 0: the unguarded kernel
                                        (256, 64, 256, None), (256, 320, 512, "mixed"), (512, 128, 256, "max"),
                                        # the ping-pong kernel: 1, 2, 3 chunks (prologue / ring edges), a
                                        # deep ring, extremes through every slot
                                        (256, 192, 256, None), (768, 4096, 512, None), (512, 4032, 256, "min"), (256, 256, 512, "min"),
                                        (256, 1216, 768, "max"),
                                        # K % 128 == 0: the 128-deep ping-pong (two-slot ring): 1, 2, 3,
                                        # 9 chunks, extremes through both slots of every region
                                        (256, 128, 256, "mixed"), (256, 384, 256, None), (512, 1152, 256, "min"),
                                        (256, 2048, 256, "max"),
                                        # K % 16 == 0 but not % 64, ragged N: vector loads with a tail
                                        (256, 80, 272, None)])
def test_mat_mult_q7_bitexact(dsp, torch_gpu, ref, m, k, n, fill):
    """arm_mat_mult_q7 (arm_mat_mult_q7.c:689-790) on one i8 MFMA plane vs the reference build bit
    for bit: extremes -128 / 127 (saturating both ways), K up to 65535 (the q31 sum at its
    largest magnitude), ragged and whole tiles.  The reference keeps its output
    row offset in a uint16_t (`i = i + numColsB`, :704,:782), so for numRows * numCols > 65536 it
    writes later rows over earlier ones; there the product follows the documented contract (every
    element at its row-major place) and is compared with the exact formula, and with the reference
    on the rows it still places correctly."""
    rng = np.random.default_rng(m + 7 * k + 13 * n)
    a, b = _q7_operands(rng, m, k, n, fill)
    st, got = dsp.arm_mat_mult_fixed("q7", a, b)
    assert st == 0
    assert got.tobytes() == _q7_exact(a, b).tobytes(), np.argwhere(got != _q7_exact(a, b))[:5]
    rows = min(m, 65536 // n)                     # rows whose uint16_t offset does not wrap
    st_r, want = ref.mat_mult_fixed("q7", a[:rows], b)
    assert st_r == 0
    assert got[:rows].tobytes() == want.tobytes(), np.argwhere(got[:rows] != want)[:5]


def test_mat_mult_q7_batch_and_multi(dsp, torch_gpu, ref):
    """arm_mat_mult_q7_batch (guarded and unguarded shapes, 3 matrices) and
    arm_mat_mult_q7_batch_multi (two ragged shards per device) against the reference build, plus a
    1024^3 x 4 batch against exact int64 products (the bench shape)."""
    torch = torch_gpu
    rng = np.random.default_rng(5)
    for (m, k, n) in ((96, 200, 80), (256, 256, 256)):
        a = rng.integers(-128, 128, (3, m, k)).astype(np.int8)
        b = rng.integers(-128, 128, (3, k, n)).astype(np.int8)
        A, B = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
        Cm = torch.empty((3, m, n), dtype=torch.int8, device="cuda")
        dsp.mat_mult_batch(A, B, Cm)
        got = Cm.cpu().numpy()
        for i in range(3):
            assert got[i].tobytes() == _q7_exact(a[i], b[i]).tobytes(), (m, i)
            assert got[i, :64].tobytes() == ref.mat_mult_fixed("q7", a[i, :64], b[i])[1].tobytes(), (m, i)
    ndev = dsp.device_count()
    m, k, n = 70, 90, 50
    shards, host = [], []
    for s in range(2 * ndev):
        cnt = 2 + s
        a = rng.integers(-128, 128, (cnt, m, k)).astype(np.int8)
        b = rng.integers(-128, 128, (cnt, k, n)).astype(np.int8)
        dev = f"cuda:{s % ndev}"
        shards.append((torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev),
                       torch.empty((cnt, m, n), dtype=torch.int8, device=dev)))
        host.append((a, b))
    dsp.mat_mult_batch_multi(shards)
    for (a, b), (_, _, c) in zip(host, shards):
        got = c.cpu().numpy()
        for i in range(a.shape[0]):
            assert got[i].tobytes() == ref.mat_mult_fixed("q7", a[i], b[i])[1].tobytes()
    a = rng.integers(-128, 128, (4, 1024, 1024)).astype(np.int8)
    b = rng.integers(-128, 128, (4, 1024, 1024)).astype(np.int8)
    A, B = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    Cm = torch.empty((4, 1024, 1024), dtype=torch.int8, device="cuda")
    dsp.mat_mult_batch(A, B, Cm)
    s = np.matmul(a.astype(np.int32), b.astype(np.int32))
    want = np.clip(s >> 7, -128, 127).astype(np.int8)
    assert Cm.cpu().numpy().tobytes() == want.tobytes()


def test_mat_mult_q7_pingpong_repeatable(dsp, torch_gpu):
    """The ping-pong kernel's LDS ordering (DMA wait + barrier before a read, refill two phases
    after the last read) screened by repetition: 1024^3 x 16 (one workgroup per CU) run six times
    must give the same words every time, and two of the matrices the exact int64 products."""
    torch = torch_gpu
    rng = np.random.default_rng(61)
    a = rng.integers(-128, 128, (16, 1024, 1024)).astype(np.int8)
    b = rng.integers(-128, 128, (16, 1024, 1024)).astype(np.int8)
    A, B = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    Cm = torch.empty((16, 1024, 1024), dtype=torch.int8, device="cuda")
    dsp.mat_mult_batch(A, B, Cm)
    first = Cm.clone()
    for _ in range(5):
        Cm.fill_(0)
        dsp.mat_mult_batch(A, B, Cm)
        assert torch.equal(Cm, first)
    got = first.cpu().numpy()
    for i in (0, 11):
        s = np.matmul(a[i].astype(np.int32), b[i].astype(np.int32))
        assert got[i].tobytes() == np.clip(s >> 7, -128, 127).astype(np.int8).tobytes(), i


@pytest.mark.parametrize("batch,m,k,n", [(1, 4608, 256, 4096), (81, 512, 512, 512)])
def test_mat_mult_q7_pp2_multitile(dsp, torch_gpu, batch, m, k, n):
    """The 128-deep ping-pong kernel with several tiles per persistent workgroup, so the chunk
    stream (and its refills: B one chunk ahead, A0 two) runs across tile boundaries: 288 tiles
    (XCD-contiguous runs, tiles % 8 == 0) and 81 x 4 = 324 tiles (round robin), against exact
    products (float64 matmul: |sum| < 2^53)."""
    torch = torch_gpu
    rng = np.random.default_rng(batch + m + k)
    a = rng.integers(-128, 128, (batch, m, k)).astype(np.int8)
    b = rng.integers(-128, 128, (batch, k, n)).astype(np.int8)
    A, B = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    Cm = torch.empty((batch, m, n), dtype=torch.int8, device="cuda")
    dsp.mat_mult_batch(A, B, Cm)
    s = np.matmul(a.astype(np.float64), b.astype(np.float64)).astype(np.int64)
    want = np.clip(s >> 7, -128, 127).astype(np.int8)
    got = Cm.cpu().numpy()
    assert got.tobytes() == want.tobytes(), np.argwhere(got != want)[:5]
