"""MFCC f32: arm_mfcc_f32 = normalise, window, RFFT, |X|, Mel,
log, DCT (Source/TransformFunctions/arm_mfcc_f32.c:83-160).

CPU: the oracle restatement is bit-identical to the reference build on the suite's inputs
and seeded frames (tests/golden/mfcc_f32.npz, produced by oracle/_ref) and meets the
reference suite's own thresholds against its double-precision patterns
(Testing/Source/Tests/MFCCF32.cpp:7-13: SNR >= 115 dB, |err| <= 1e-5 + 1.2e-3*|ref|).

GPU: every stage is the reference's arithmetic in the reference's order, and the one libm
call, logf (arm_vlog_f32.c:110), is the host glibc 2.35 logf restated for the device
(csrc/host_logf.hpp; tools/logf_check.cpp proves it equal to the host's on all 2^32 inputs), so
the coefficients are held BIT-EXACT to the reference build, plus the suite's thresholds
against the patterns.
"""
import numpy as np
import pytest

import mfcc_cfg
from metrics import snr_db

SUITE_N = (256, 512, 1024)


def _close(got, want):
    """Bit-exact, elementwise (NaN patterns included)."""
    return np.ascontiguousarray(got, np.float32).view(np.uint32) == np.ascontiguousarray(want, np.float32).view(np.uint32)


# ------------------------------------------------------------------ CPU (oracle)
@pytest.mark.parametrize("n", SUITE_N)
def test_oracle_bitexact_vs_reference_fixture(oracle, n):
    g = mfcc_cfg.golden()
    got = oracle.mfcc(mfcc_cfg.suite_cfg(g, n), g[f"frames_{n}"])
    assert got.tobytes() == g[f"out_{n}"].tobytes()


@pytest.mark.parametrize("n", SUITE_N)
@pytest.mark.parametrize("kind", ["Noise", "Sine"])
def test_oracle_meets_reference_suite_thresholds(oracle, n, kind):
    g = mfcc_cfg.golden()
    got = oracle.mfcc(mfcc_cfg.suite_cfg(g, n), g[f"input_{kind}_{n}"])[0]
    ref = g[f"ref_{kind}_{n}"]
    assert snr_db(ref, got) >= 115
    assert np.all(np.abs(got - ref) <= 1e-5 + 1.2e-3 * np.abs(ref))


def test_oracle_matches_reference_build_random_configs(oracle, ref):
    for n in (32, 128, 2048, 4096):
        cfg = mfcc_cfg.make_cfg(n)
        x = np.random.default_rng(n).uniform(-1, 1, (3, n)).astype(np.float32)
        assert oracle.mfcc(cfg, x).tobytes() == ref.mfcc(cfg, x).tobytes(), n


def test_host_libm_logf_is_the_restated_one():
    """The precondition of MFCC f32 bit-exactness on this host (reported, never a failure of
    the product: a different libm makes the GPU tests skip with "libm differs")."""
    ok, bad, glibc = mfcc_cfg.host_libm_status()
    if not ok:
        pytest.skip(f"host libm differs ({glibc}): {bad} sampled mismatches")


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n", SUITE_N)
def test_gpu_dropin_vs_reference_fixture(dsp, torch_gpu, n):
    g = mfcc_cfg.golden()
    cfg = mfcc_cfg.suite_cfg(g, n)
    m = dsp.MfccF32(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
    want = g[f"out_{n}"]
    got = np.stack([m(f) for f in g[f"frames_{n}"]])
    for i, kind in enumerate(("Noise", "Sine")):
        r = g[f"ref_{kind}_{n}"]
        assert snr_db(r, got[i]) >= 115
        assert np.all(np.abs(got[i] - r) <= 1e-5 + 1.2e-3 * np.abs(r))
    mfcc_cfg.assert_parity(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("n", (32, 64, 128, 256, 512, 1024, 2048, 4096))
def test_gpu_batch_vs_reference_build(dsp, torch_gpu, ref, n):
    cfg = mfcc_cfg.make_cfg(n)
    rng = np.random.default_rng(7 * n)
    frames = rng.uniform(-1, 1, (37, n)).astype(np.float32)
    frames[3] = 0.0                       # max == 0: no normalisation (arm_mfcc_f32.c:102)
    frames[4] *= 1e-30                    # tiny, denormal-range products
    frames[5] = np.sin(np.arange(n) * 0.3).astype(np.float32) * 1e4
    want = ref.mfcc(cfg, frames)
    m = dsp.MfccF32(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
    got = m.batch(torch_gpu.from_numpy(frames.copy()).cuda()).cpu().numpy()
    # the batch equals the drop-in call frame by frame, bit for bit (no libm involved)
    single = np.stack([m(f) for f in frames[:6]])
    assert single.tobytes() == got[:6].tobytes()
    mfcc_cfg.assert_parity(got, want, suite_tolerance=False)


@pytest.mark.gpu
def test_gpu_batch_device_tables_and_content_cache(dsp, torch_gpu, ref):
    """Tables as device tensors; then a host table buffer reused with new contents must be
    re-uploaded (the device copy is cached by content, not by pointer)."""
    n = 512
    cfg = mfcc_cfg.make_cfg(n)
    frames = np.random.default_rng(1).uniform(-1, 1, (8, n)).astype(np.float32)
    dev = {k: torch_gpu.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in cfg.items() if k != "fftLen"}
    m = dsp.MfccF32(n, dev["dct"], dev["pos"], dev["len"], dev["coefs"], dev["window"])
    got = m.batch(torch_gpu.from_numpy(frames.copy()).cuda()).cpu().numpy()
    mfcc_cfg.assert_parity(got, ref.mfcc(cfg, frames), suite_tolerance=False)
    host = {k: np.ascontiguousarray(v).copy() for k, v in cfg.items() if k != "fftLen"}
    m2 = dsp.MfccF32(n, host["dct"], host["pos"], host["len"], host["coefs"], host["window"])
    a = m2.batch(torch_gpu.from_numpy(frames.copy()).cuda()).cpu().numpy()
    m2._t[4][0][:] = np.hanning(n).astype(np.float32)            # same buffer, new window
    cfg2 = dict(cfg, window=m2._t[4][0].copy())
    b = m2.batch(torch_gpu.from_numpy(frames.copy()).cuda()).cpu().numpy()
    assert not np.array_equal(a, b)
    mfcc_cfg.assert_parity(np.stack([a, b]), np.stack([ref.mfcc(cfg, frames), ref.mfcc(cfg2, frames)]),
                           suite_tolerance=False)


@pytest.mark.gpu
def test_gpu_unfused_path_more_filters_than_half_spectrum(dsp, torch_gpu, ref):
    """nbMelFilters > fftLen/2 takes the three-launch path (pre, RFFT, post)."""
    n, nb_mel = 64, 40
    cfg = {"fftLen": n, "pos": np.array([i % 30 for i in range(nb_mel)], np.uint32),
           "len": np.full(nb_mel, 2, np.uint32),
           "coefs": np.random.default_rng(3).uniform(0, 1, 2 * nb_mel).astype(np.float32),
           "dct": np.random.default_rng(4).uniform(-0.3, 0.3, (13, nb_mel)).astype(np.float32),
           "window": np.hanning(n).astype(np.float32)}
    frames = np.random.default_rng(5).uniform(-1, 1, (9, n)).astype(np.float32)
    m = dsp.MfccF32(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
    got = m.batch(torch_gpu.from_numpy(frames.copy()).cuda()).cpu().numpy()
    mfcc_cfg.assert_parity(got, ref.mfcc(cfg, frames), suite_tolerance=False)
