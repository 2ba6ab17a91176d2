"""Multirate FIR: arm_fir_decimate_{f32,q15,fast_q15,q31,fast_q31} and
arm_fir_interpolate_{f32,q15,q31} (+ their inits and the batched device API).

CPU: the oracle restatement (oracle/src/oracle_multirate.c) equals the reference build
(oracle/_ref, Source/FilteringFunctions/arm_fir_decimate_*.c / arm_fir_interpolate_*.c) bit
for bit: outputs of consecutive calls and the final state buffer, over tap counts, factors and
block sizes that hit the reference's unrolled and remainder loops, full-range fixed-point data
(wrap / saturation) and the init length checks.
GPU: the product (drop-in through host buffers, and the batched device API over several
streams and two calls each) equals the reference build bit for bit.
"""
import ctypes as C

import numpy as np
import pytest

import refs
from cmsisdsp_amd import _abi

DECIM = ["decimate_f32", "decimate_q15", "decimate_fast_q15", "decimate_q31", "decimate_fast_q31"]
INTERP = ["interpolate_f32", "interpolate_q15", "interpolate_q31"]
# (taps, factor, block sizes): decimators need blockSize % M == 0, interpolators numTaps % L == 0
DCASES = [(128, 2, [4096, 4096]), (29, 3, [33, 66, 3]), (1, 1, [16, 5]), (7, 8, [64, 8]), (130, 5, [100, 200]),
          (64, 255, [510]), (3, 4, [4, 8, 12]), (40, 1, [37, 100])]
ICASES = [(128, 2, [4096, 100]), (30, 3, [33, 7, 1]), (1, 1, [16, 5]), (64, 8, [64, 8]), (125, 5, [100, 3]),
          (255, 255, [20]), (12, 4, [9, 13]), (40, 1, [37, 100])]


def data(kind, n, rng, dist="full"):
    if kind == "f32":
        return rng.standard_normal(n).astype(np.float32)
    info = np.iinfo(refs.DTYPE[kind])
    if dist == "min":
        return np.full(n, info.min, refs.DTYPE[kind])
    return rng.integers(info.min, info.max, n, endpoint=True).astype(refs.DTYPE[kind])


def case(fn, taps, blocks, seed, dist="full"):
    kind = fn.split("_")[-1]
    rng = np.random.default_rng(seed)
    c = data(kind, taps, rng, dist)
    if kind == "f32":
        c = (c / np.sqrt(taps)).astype(np.float32)
    return c, [data(kind, b, rng, dist) for b in blocks]


def same(a, b):
    sa, ya, ta = a
    sb, yb, tb = b
    assert sa == sb
    assert len(ya) == len(yb)
    for u, v in zip(ya, yb):
        assert u.tobytes() == v.tobytes()
    assert ta.tobytes() == tb.tobytes()


# ------------------------------------------------------------------ CPU: oracle == reference
@pytest.mark.parametrize("fn", DECIM)
@pytest.mark.parametrize("taps,M,blocks", DCASES)
def test_decimate_oracle_equals_reference(oracle, ref, fn, taps, M, blocks):
    c, xs = case(fn, taps, blocks, taps * 7 + M)
    same(oracle.multirate(fn, M, c, xs), ref.multirate(fn, M, c, xs))


@pytest.mark.parametrize("fn", INTERP)
@pytest.mark.parametrize("taps,L,blocks", ICASES)
def test_interpolate_oracle_equals_reference(oracle, ref, fn, taps, L, blocks):
    c, xs = case(fn, taps, blocks, taps * 5 + L)
    same(oracle.multirate(fn, L, c, xs), ref.multirate(fn, L, c, xs))


@pytest.mark.parametrize("fn", [f for f in DECIM + INTERP if not f.endswith("f32")])
def test_multirate_extreme_words(oracle, ref, fn):
    """All-minimum samples and taps: the q63 / q31 accumulators wrap, outputs saturate."""
    factor, taps = (2, 32) if fn.startswith("decimate") else (4, 32)
    c, xs = case(fn, taps, [64, 64], 1, dist="min")
    same(oracle.multirate(fn, factor, c, xs), ref.multirate(fn, factor, c, xs))


@pytest.mark.parametrize("fn", ["decimate_f32", "decimate_q15", "interpolate_q31"])
def test_multirate_init_length_error(oracle, ref, fn):
    """blockSize % M != 0 (decimators) / numTaps % L != 0 (interpolators): ARM_MATH_LENGTH_ERROR."""
    c, xs = case(fn, 30, [35], 2)
    for h in (oracle, ref):
        st, outs, _ = h.multirate(fn, 4, c, xs, block_size=35)
        assert st == _abi.ARM_MATH_LENGTH_ERROR and outs == []


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module")
def product(dsp):
    return refs.Host(dsp.lib, "")


@pytest.mark.gpu
@pytest.mark.parametrize("fn", DECIM + INTERP)
def test_multirate_dropin_bitexact(product, torch_gpu, ref, fn):
    for taps, factor, blocks in (DCASES if fn.startswith("decimate") else ICASES):
        c, xs = case(fn, taps, blocks, taps + factor)
        same(product.multirate(fn, factor, c, xs), ref.multirate(fn, factor, c, xs))


@pytest.mark.gpu
@pytest.mark.parametrize("fn", DECIM + INTERP)
@pytest.mark.parametrize("taps,factor,block", [(128, 4, 4096), (31, 3, 999), (256, 2, 2050)])
def test_multirate_batch_bitexact(dsp, torch_gpu, ref, fn, taps, factor, block):
    """Batched device API: 5 streams, two consecutive calls each, history carried in d_hist."""
    torch = torch_gpu
    decim = fn.startswith("decimate")
    if not decim:
        taps -= taps % factor
    kind = fn.split("_")[-1]
    tdt = {"f32": torch.float32, "q15": torch.int16, "q31": torch.int32}[kind]
    batch = 5
    c, _ = case(fn, taps, [1], taps * 3 + factor)
    streams = [case(fn, taps, [block, block], 100 + i)[1] for i in range(batch)]
    dc = torch.from_numpy(c.copy()).cuda()
    if decim:
        S = _abi.arm_fir_decimate_instance(M=factor, numTaps=taps, pCoeffs=dc.data_ptr(), pState=None)
        H, nout = taps - 1, block // factor
    else:
        S = _abi.arm_fir_interpolate_instance(L=factor, phaseLength=taps // factor, pCoeffs=dc.data_ptr(),
                                              pState=None)
        H, nout = taps // factor - 1, block * factor
    hist = torch.zeros((batch, max(H, 1)), dtype=tdt, device="cuda")
    f = getattr(dsp.lib, f"arm_fir_{fn}_batch")
    got = []
    for k in range(2):
        src = torch.from_numpy(np.stack([streams[i][k] for i in range(batch)])).cuda()
        dst = torch.empty((batch, nout), dtype=tdt, device="cuda")
        st = f(C.byref(S), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), block, batch,
               C.c_void_p(hist.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert st == 0, dsp.last_error()
        got.append(dst.cpu().numpy())
    h = hist.cpu().numpy()
    for i in range(batch):
        st, want, state = ref.multirate(fn, factor, c, streams[i])
        assert st == 0
        for k in range(2):
            assert got[k][i].tobytes() == want[k].tobytes(), (i, k)
        assert h[i, :H].tobytes() == state[:H].tobytes()


@pytest.mark.gpu
def test_cmsisdsp_module_multirate_and_q7(torch_gpu, ref):
    """The cmsisdsp-compatible module with the reference binding's call shapes
    (cmsisdsp_filtering.c: init "OhiOO" / "OihOO", blockSize = len(pState) - len(pCoeffs) + 1)."""
    import cmsisdsp as d
    rng = np.random.default_rng(5)
    c = (rng.standard_normal(24) / 5).astype(np.float32)
    x = rng.standard_normal(96).astype(np.float32)
    S = d.arm_fir_decimate_instance_f32()
    assert d.arm_fir_decimate_init_f32(S, 24, 4, c, np.zeros(24 + 96 - 1)) == 0
    want = ref.multirate("decimate_f32", 4, c, [x])[1][0]
    assert d.arm_fir_decimate_f32(S, x).tobytes() == want.tobytes()
    ci = rng.integers(-32768, 32767, 24).astype(np.int16)
    xi = rng.integers(-32768, 32767, 40).astype(np.int16)
    S = d.arm_fir_interpolate_instance_q15()
    assert d.arm_fir_interpolate_init_q15(S, 3, 24, ci, np.zeros(24 + 40 - 1)) == 0
    want = ref.multirate("interpolate_q15", 3, ci, [xi], block_size=40)[1][0]
    assert d.arm_fir_interpolate_q15(S, xi).tobytes() == want.tobytes()
    a7 = rng.integers(-128, 127, 50).astype(np.int8)
    b7 = rng.integers(-128, 127, 9).astype(np.int8)
    assert d.arm_conv_q7(a7, 50, b7, 9).tobytes() == ref.conv("q7", a7, b7).tobytes()
    F = d.arm_fir_instance_q7()
    d.arm_fir_init_q7(F, 9, b7, np.zeros(9 + 50 - 1))
    want = ref.fir("q7", b7, [a7])[0][0]
    assert d.arm_fir_q7(F, a7).tobytes() == want.tobytes()
