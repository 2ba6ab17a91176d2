"""MFCC q15 (the q15 caller of the q15 RFFT): arm_mfcc_q15 = normalise (absmax, divide_q15,
scale_q15), window, RFFT q15, |X| (sqrt_q31 >> 16), Mel (q63 sums), scale_q31, log_q31,
offset, >> 19 truncated to q15, DCT with arm_mat_vec_mult_q15's int32-wrapped column pairs
(Source/TransformFunctions/arm_mfcc_q15.c:96-228).  Integer throughout: bit-exact everywhere.

CPU: the oracle restatement (oracle/src/oracle_mfcc_fixed.c) is bit-identical to the reference
build on the suite's inputs plus seeded and edge frames (tests/golden/mfcc_q15.npz, made by
tools/make_golden.py mfcc_q15 from oracle/_ref) and meets the reference suite's thresholds
against its patterns (Testing/Source/Tests/MFCCQ15.cpp:7-8: SNR >= 34 dB, |err| <= 30).
GPU: drop-in and batched paths bit-exact against the fixture and the reference build.
"""
import numpy as np
import pytest

import mfcc_cfg
from metrics import snr_db

SUITE_N = (256, 512, 1024)
GOLDEN = mfcc_cfg.GOLDEN.replace("mfcc_f32.npz", "mfcc_q15.npz")


def golden():
    return dict(np.load(GOLDEN))


def suite_cfg(g, n):
    return {"fftLen": n, "dct": g["dct"], "pos": g[f"pos_{n}"], "len": g[f"len_{n}"], "coefs": g[f"coefs_{n}"],
            "window": g[f"window_{n}"]}


def q15(a):
    return np.clip(np.round(np.asarray(a, np.float64) * 2.0**15), -2**15, 2**15 - 1).astype(np.int16)


def make_cfg_q15(n):
    c = mfcc_cfg.make_cfg(n)
    return {"fftLen": n, "dct": q15(c["dct"]), "pos": c["pos"], "len": c["len"], "coefs": q15(c["coefs"]),
            "window": q15(c["window"])}


def frames_for(n, rows, seed):
    rng = np.random.default_rng(seed)
    f = rng.integers(-2**14, 2**14, (rows, n)).astype(np.int16)
    f[1] = 0
    f[2] = rng.integers(-3, 4, n)
    f[3, 5] = -2**15
    f[4] = (np.sin(np.arange(n) * 0.21) * 2**13).astype(np.int16)
    # max |x| == 1: the only frame for which arm_scale's shift count reaches the word size
    # (the reference's undefined shift, taken mod 32 on the x86 host)
    f[5] = rng.integers(-1, 2, n)
    f[5, 3] = -1
    return f


# ------------------------------------------------------------------ CPU (oracle)
@pytest.mark.parametrize("n", SUITE_N)
def test_oracle_bitexact_vs_reference_fixture(oracle, n):
    g = golden()
    got = oracle.mfcc_q15(suite_cfg(g, n), g[f"frames_{n}"])
    assert got.tobytes() == g[f"out_{n}"].tobytes()


@pytest.mark.parametrize("n", SUITE_N)
@pytest.mark.parametrize("kind", ["Noise", "Sine"])
def test_oracle_meets_reference_suite_thresholds(oracle, n, kind):
    g = golden()
    got = oracle.mfcc_q15(suite_cfg(g, n), g[f"input_{kind}_{n}"])[0]
    ref = g[f"ref_{kind}_{n}"]
    assert snr_db(ref.astype(np.float64), got.astype(np.float64)) >= 34
    assert np.all(np.abs(got.astype(np.int32) - ref) <= 30)


def test_oracle_matches_reference_build_generated_configs(oracle, ref):
    for n in (32, 64, 128, 2048, 4096):
        cfg = make_cfg_q15(n)
        x = frames_for(n, 6, n)
        assert oracle.mfcc_q15(cfg, x).tobytes() == ref.mfcc_q15(cfg, x).tobytes(), n


def test_oracle_dct_pairs_wrap_like_the_reference(oracle, ref):
    """Extreme DCT rows (all -32768) over 21 Mel filters (an odd column count): the pair /
    quad / tail split of arm_mat_vec_mult_q15's __SMLALD columns (rows in groups of four pair
    columns up to 20, the 13th row pairs within column quads) against floor log values."""
    n = 256
    g = golden()
    cfg = suite_cfg(g, n)
    cfg["dct"] = np.full((13, 21), -32768, np.int16)
    cfg["pos"], cfg["len"] = np.append(cfg["pos"], 5).astype(np.uint32), np.append(cfg["len"], 1).astype(np.uint32)
    cfg["coefs"] = np.append(cfg["coefs"], 100).astype(np.int16)
    x = np.zeros((2, n), np.int16)
    x[1, :4] = 1
    assert oracle.mfcc_q15(cfg, x).tobytes() == ref.mfcc_q15(cfg, x).tobytes()


def test_oracle_matches_reference_build_edge_filters(oracle, ref):
    for n in (256, 1024):
        rng = np.random.default_rng(n + 7)
        base = make_cfg_q15(n)
        x = frames_for(n, 6, 5 * n)
        for pos, ln in mfcc_cfg.edge_filterbanks(n, rng):
            cfg = dict(base, pos=pos, len=ln,
                       coefs=rng.integers(-2**15, 2**15, int(ln.sum()), dtype=np.int64).astype(np.int16),
                       dct=rng.integers(-2**15, 2**15, (4, len(pos)), dtype=np.int64).astype(np.int16))
            assert oracle.mfcc_q15(cfg, x).tobytes() == ref.mfcc_q15(cfg, x).tobytes(), (n, pos, ln)


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("n", SUITE_N)
def test_gpu_dropin_and_batch_vs_reference_fixture(dsp, torch_gpu, n):
    g = golden()
    cfg = suite_cfg(g, n)
    m = dsp.MfccQ15(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
    want = g[f"out_{n}"]
    got = np.stack([m(f) for f in g[f"frames_{n}"]])
    assert got.tobytes() == want.tobytes(), np.argwhere(got != want)[:5]
    b = m.batch(torch_gpu.from_numpy(g[f"frames_{n}"].copy()).cuda()).cpu().numpy()
    assert b.tobytes() == want.tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("n", (32, 64, 128, 256, 512, 1024, 2048, 4096))
def test_gpu_batch_vs_reference_build(dsp, torch_gpu, ref, n):
    cfg = make_cfg_q15(n)
    frames = frames_for(n, 37, 13 * n)
    want = ref.mfcc_q15(cfg, frames)
    m = dsp.MfccQ15(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
    got = m.batch(torch_gpu.from_numpy(frames.copy()).cuda()).cpu().numpy()
    assert got.tobytes() == want.tobytes(), (n, np.argwhere(got != want)[:5])


@pytest.mark.gpu
def test_gpu_dct_pair_wrap(dsp, torch_gpu, ref):
    n = 256
    g = golden()
    cfg = suite_cfg(g, n)
    cfg["dct"] = np.full((13, 21), -32768, np.int16)
    cfg["pos"], cfg["len"] = np.append(cfg["pos"], 5).astype(np.uint32), np.append(cfg["len"], 1).astype(np.uint32)
    cfg["coefs"] = np.append(cfg["coefs"], 100).astype(np.int16)
    x = np.zeros((2, n), np.int16)
    x[1, :4] = 1
    m = dsp.MfccQ15(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
    got = m.batch(torch_gpu.from_numpy(x.copy()).cuda()).cpu().numpy()
    assert got.tobytes() == ref.mfcc_q15(cfg, x).tobytes()


@pytest.mark.gpu
@pytest.mark.parametrize("n", (256, 512, 1024, 4096))
def test_gpu_filters_at_spectrum_edges(dsp, torch_gpu, ref, n):
    """Filters on bins 0 and fftLen/2, an empty one, a narrow odd-based range, the whole half
    spectrum: the back end computes only the magnitudes in the filters' bin range."""
    rng = np.random.default_rng(n + 7)
    base = make_cfg_q15(n)
    frames = frames_for(n, 9, 3 * n)
    for pos, ln in mfcc_cfg.edge_filterbanks(n, rng):
        nb = len(pos)
        cfg = dict(base, pos=pos, len=ln,
                   coefs=rng.integers(-2**15, 2**15, int(ln.sum()), dtype=np.int64).astype(np.int16),
                   dct=rng.integers(-2**15, 2**15, (4, nb), dtype=np.int64).astype(np.int16))
        want = ref.mfcc_q15(cfg, frames)
        m = dsp.MfccQ15(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
        got = m.batch(torch_gpu.from_numpy(frames.copy()).cuda()).cpu().numpy()
        assert got.tobytes() == want.tobytes(), (n, pos, ln, np.argwhere(got != want)[:5])
