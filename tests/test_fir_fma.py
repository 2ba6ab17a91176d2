"""arm_fir_f32_batch_fma — the opt-in tolerance path of the batched f32 FIR.

Every output sums its taps in the reference's order (arm_fir_f32.c:911-1280), but each MAC is
one fused multiply-add, so the result is held to tolerances instead of bits:
  * the reference suite's own thresholds on its FIR F32 patterns (FIRF32.cpp:5,13: SNR >= 120
    dB and |out - ref| <= 3e-5 |ref|), replaying the suite's two-block call sequence;
  * per element against a float64 evaluation: |y - y64| <= numTaps * 2^-24 * sum_k |x_k b_k|
    (the recursive-summation bound of a K-term f32 sum; an fma chain satisfies it);
  * a negative control: the bit-exact path's outputs are within the same bound but the FMA
    path must differ from them somewhere (proving the FMA kernel ran).
"""
import numpy as np
import pytest

import metrics
from test_golden import pat  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def _fir64(c, blocks):
    """float64 FIR over consecutive blocks (zero initial state) + the sum of |x b| per output."""
    x = np.concatenate(blocks).astype(np.float64)
    T = len(c)
    s = np.concatenate([np.zeros(T - 1), x])
    w = np.lib.stride_tricks.sliding_window_view(s, T)          # w[n] = s[n .. n+T-1]
    cc = c.astype(np.float64)        # pCoeffs time-reversed (arm_fir_f32.c): y[n] = sum_k s[n+k] c[k]
    return w @ cc, np.abs(w) @ np.abs(cc)


def _run(dsp, torch, kind, c, blocks_per_filter):
    from test_gpu_rfft_fir_mat import _fir_batched
    return _fir_batched(dsp, torch, kind, c, blocks_per_filter)


def test_fma_reference_suite_thresholds(dsp, torch_gpu, pat):  # noqa: F811
    cfg = pat["fir_f32_configs"].reshape(-1, 2)
    coefs, inp = pat["fir_f32_coefs"], pat["fir_f32_input"]
    outs, off = [], 0
    for block, taps in cfg:
        c = coefs[off:off + taps]
        off += taps
        got, _ = _run(dsp, torch_gpu, "f32_fma", c, [[inp[:block], inp[block:2 * block]]])
        outs += [got[0][0], got[1][0]]
    got = np.concatenate(outs)
    want = pat["fir_f32_refs"]
    assert metrics.snr_db(want, got) >= metrics.FIR_TOL["f32"]["snr"]
    assert metrics.rel_error(got, want, metrics.FIR_TOL["f32"]["rel"])


@pytest.mark.parametrize("taps,block", [(128, 4096), (29, 32), (1, 64), (255, 1000), (256, 1500), (257, 777), (64, 5000),
                                        (7, 1023), (1024, 3000), (2047, 2500)])
def test_fma_elementwise_bound_vs_float64(dsp, torch_gpu, taps, block):
    rng = np.random.default_rng(taps + block)
    batch = 3
    c = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
    blocks = [[rng.uniform(-1, 1, block).astype(np.float32) for _ in range(2)] for _ in range(batch)]
    got, hist = _run(dsp, torch_gpu, "f32_fma", c, blocks)
    exact, _ = _run(dsp, torch_gpu, "f32", c, blocks)
    differs = False
    for f in range(batch):
        y = np.concatenate([got[0][f], got[1][f]]).astype(np.float64)
        y64, mag = _fir64(c, blocks[f])
        assert np.all(np.abs(y - y64) <= taps * 2.0 ** -24 * mag + 1e-30), f
        differs |= np.concatenate([exact[0][f], exact[1][f]]).tobytes() != y.astype(np.float32).tobytes()
        if taps > 1:   # the state contract is the bit-exact path's: the last numTaps-1 inputs
            assert hist[f].tobytes() == np.concatenate(blocks[f])[-(taps - 1):].tobytes()
    assert differs or taps == 1, "the FMA path returned the bit-exact path's words everywhere"
