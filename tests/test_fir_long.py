"""Long filters: numTaps above the 1024-tap LDS window, up to the uint16_t maximum.

The reference accepts any uint16_t numTaps (arm_fir_init_f32.c:72-95, filtering_functions.h:
58-98) and its scalar loops have no limit (arm_fir_f32.c:911-1280, arm_fir_q15.c:458-726,
arm_fir_q31.c, arm_fir_fast_q15.c, arm_fir_fast_q31.c, arm_fir_q7.c:446-560).  The product
runs such filters in 1024-tap segments with the accumulators carried in registers (fir.hip,
fir_f32_kernel<.., LONG> and the segment loops of the fixed-point kernels), so the f32 sum
keeps the reference's sequential tap order.  The multirate filters fall back to a direct
kernel when the window does not fit the LDS image (fir_mr_direct_kernel).
"""
import numpy as np
import pytest

import refs
from test_gpu_rfft_fir_mat import FIR_KINDS, _fir_batched
from test_multirate import case, same

LONG_TAPS = [1025, 2047, 4096, 65535]


def _data(kind, taps, blocks, seed):
    rng = np.random.default_rng(seed)
    if kind == "f32":
        c = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
        xs = [rng.uniform(-1, 1, b).astype(np.float32) for b in blocks]
        return c, xs
    bits, dt = {"q15": (15, np.int16), "q31": (31, np.int32), "q7": (7, np.int8)}[kind.split("_")[-1]]
    lo, hi = -(1 << bits), (1 << bits) - 1
    c = rng.integers(lo, hi, taps, endpoint=True).astype(dt)
    return c, [rng.integers(lo, hi, b, endpoint=True).astype(dt) for b in blocks]


def _taps_for(kind, taps):
    # q15 filters need an even numTaps (arm_fir_init_q15.c:95-106): 1025 -> 1026, 65535 -> 65534
    if not kind.endswith("q15") or taps % 2 == 0:
        return taps
    return taps + 1 if taps < 65535 else taps - 1


# ------------------------------------------------------------------ CPU: oracle == reference
@pytest.mark.parametrize("kind", FIR_KINDS)
@pytest.mark.parametrize("taps", [1025, 4096])
def test_fir_long_oracle_equals_reference(oracle, ref, kind, taps):
    taps = _taps_for(kind, taps)
    c, xs = _data(kind, taps, [700, 3000], taps)
    wo, so = oracle.fir(kind, c, xs)
    wr, sr = ref.fir(kind, c, xs)
    for a, b in zip(wo, wr):
        assert a.tobytes() == b.tobytes()
    assert so.tobytes() == sr.tobytes()


# ------------------------------------------------------------------ GPU parity
@pytest.mark.gpu
@pytest.mark.parametrize("kind", FIR_KINDS)
@pytest.mark.parametrize("taps", LONG_TAPS)
def test_fir_long_batch_two_calls(dsp, torch_gpu, ref, kind, taps):
    """Two consecutive calls per filter (state carry), numTaps 1025 / 2047 / 4096 / 65535:
    a first block shorter than numTaps (the new history then reaches the old one), a second
    spanning several 2048-output chunks."""
    taps = _taps_for(kind, taps)
    block = 300 if taps > 10000 else 2500
    batch = 2 if taps > 10000 else 3
    per = [_data(kind, taps, [block, block], taps * 3 + f) for f in range(batch)]
    c = per[0][0]
    blocks = [p[1] for p in per]
    got, hist = _fir_batched(dsp, torch_gpu, kind, c, blocks)
    for f in range(batch):
        want, state = ref.fir(kind, c, blocks[f])
        for k in range(2):
            assert got[k][f].tobytes() == want[k].tobytes(), (f, k)
        assert hist[f].tobytes() == state[:taps - 1].tobytes()


@pytest.mark.gpu
def test_fir_long_f32_extreme_tail(dsp, torch_gpu, ref):
    """numTaps % 8 tail taps in the last segment and a 1-tap last segment (1025 = 1024 + 1),
    blocks not a multiple of 8 and a ragged last chunk."""
    for taps, block in ((1025, 2049), (3079, 4103), (2048, 7)):
        c, xs = _data("f32", taps, [block, block], taps)
        got, hist = _fir_batched(dsp, torch_gpu, "f32", c, [xs])
        want, state = ref.fir("f32", c, xs)
        for k in range(2):
            assert got[k][0].tobytes() == want[k].tobytes(), (taps, block, k)
        assert hist[0].tobytes() == state[:taps - 1].tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["f32", "q15", "q31", "q7"])
def test_fir_long_dropin(dsp, torch_gpu, ref, kind):
    """Host-pointer drop-in arm_fir_* at 4096 taps over three calls: outputs and the
    caller's state buffer equal the reference's (no silent no-op above 1024 taps)."""
    taps, block = 4096, 512
    c, xs = _data(kind, taps, [block] * 3, 77)
    f = {"f32": dsp.FirF32, "q15": dsp.FirQ15, "q31": dsp.FirQ31, "q7": dsp.FirQ7}[kind](c, block)
    want, state = ref.fir(kind, c, xs)
    for x, w in zip(xs, want):
        assert f(x).tobytes() == w.tobytes()
    assert f.state.tobytes() == state.tobytes()


@pytest.mark.gpu
def test_fir_long_q15_extremes(dsp, torch_gpu, ref):
    """-32768 samples against -32768 taps over 2048 taps: the wrapping pair path in both
    segments, the int64 segment sums, the blockSize % 4 tail."""
    taps, block = 2048, 4099
    c = np.full(taps, -32768, dtype=np.int16)
    x = np.full(block, -32768, dtype=np.int16)
    got, _ = _fir_batched(dsp, torch_gpu, "q15", c, [[x]])
    want, _ = ref.fir("q15", c, [x])
    assert got[0][0].tobytes() == want[0].tobytes()


# multirate windows past the 8192-element LDS image: the direct kernel
LONG_MR = [("decimate_f32", 9000, 2, [64, 66]), ("decimate_q15", 9000, 2, [64, 66]),
           ("decimate_fast_q15", 8193, 1, [40, 17]), ("decimate_q31", 9001, 3, [63, 30]),
           ("decimate_fast_q31", 16500, 2, [50, 20]), ("interpolate_f32", 16000, 2, [40, 9]),
           ("interpolate_q15", 16000, 2, [33, 20]), ("interpolate_q31", 24000, 3, [25, 10])]


@pytest.mark.parametrize("fn,taps,factor,blocks", LONG_MR)
def test_multirate_long_oracle_equals_reference(oracle, ref, fn, taps, factor, blocks):
    c, xs = case(fn, taps, blocks, taps + factor)
    same(oracle.multirate(fn, factor, c, xs), ref.multirate(fn, factor, c, xs))


@pytest.mark.gpu
@pytest.mark.parametrize("fn,taps,factor,blocks", LONG_MR)
def test_multirate_long_dropin(dsp, torch_gpu, ref, fn, taps, factor, blocks):
    product = refs.Host(dsp.lib, "")
    c, xs = case(fn, taps, blocks, taps + factor)
    same(product.multirate(fn, factor, c, xs), ref.multirate(fn, factor, c, xs))
