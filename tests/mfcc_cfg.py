"""MFCC test configurations: the reference suite's tables (tests/golden/mfcc_f32.npz, data of
Testing/Source/Tests/mfccdata.c) and a small generator of further valid configurations
(triangular Mel filters below fftLen/2, orthonormal DCT-II, Hamming window) for the sizes
the suite does not cover.  The checkers receive the same tables, so any valid table set
exercises the same arithmetic."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mfcc_f32.npz")


def golden():
    return dict(np.load(GOLDEN))


def suite_cfg(g, n):
    return {"fftLen": n, "dct": g["dct"], "pos": g[f"pos_{n}"], "len": g[f"len_{n}"], "coefs": g[f"coefs_{n}"],
            "window": g[f"window_{n}"]}


def make_cfg(n, nb_mel=20, nb_dct=13, fs=16000.0, fmin=64.0):
    nb_mel = min(nb_mel, max(1, n // 4 - 2))
    fmax = fs / 2
    mel = lambda f: 1127.0 * np.log(1.0 + f / 700.0)       # noqa: E731
    imel = lambda m: 700.0 * (np.exp(m / 1127.0) - 1.0)    # noqa: E731
    pts = imel(np.linspace(mel(fmin), mel(fmax), nb_mel + 2))
    bins = np.clip(np.floor(n * pts / fs).astype(int), 0, n // 2 - 1)
    pos, lens, coefs = [], [], []
    for i in range(nb_mel):
        lo, mid, hi = bins[i], max(bins[i + 1], bins[i] + 1), max(bins[i + 2], bins[i] + 2)
        hi = min(hi, n // 2 - 1)
        mid = min(mid, hi)
        k = np.arange(lo, hi + 1)
        w = np.where(k <= mid, (k - lo + 1) / (mid - lo + 1), (hi - k + 1) / (hi - mid + 1))
        pos.append(lo)
        lens.append(len(k))
        coefs.append(w)
    r, c = np.meshgrid(np.arange(nb_dct), np.arange(nb_mel), indexing="ij")
    dct = np.sqrt(2.0 / nb_mel) * np.cos(np.pi / nb_mel * (c + 0.5) * r)
    dct[0] *= np.sqrt(0.5)
    win = 0.54 - 0.46 * np.cos(2 * np.pi * np.arange(n) / n)
    return {"fftLen": n, "dct": dct.astype(np.float32), "pos": np.array(pos, np.uint32),
            "len": np.array(lens, np.uint32), "coefs": np.concatenate(coefs).astype(np.float32),
            "window": win.astype(np.float32)}


_LIBM = {}


def host_libm_status(stride=4099):
    """(matches, mismatches, glibc): does the host libm logf -- the one libm call of the
    reference's MFCC f32 (arm_vlog_f32.c:110) -- equal the device restatement of glibc 2.35's
    __logf_fma (csrc/host_logf.hpp) on a strided sample of all 2^32 inputs (~1M values)?  When
    it does not, bit-exactness against the reference build is not assessable on this host
    (oracle/src/logf_probe.cpp; tools/logf_check.cpp is the exhaustive form)."""
    if "s" not in _LIBM:
        import ctypes as C
        so = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle", "_build",
                          "liblogfprobe.so")
        lib = C.CDLL(so)
        lib.logf_probe_mismatches.restype = C.c_uint64
        lib.logf_probe_mismatches.argtypes = [C.c_uint32, C.c_uint32]
        bad = int(lib.logf_probe_mismatches(stride, 17))
        try:
            glibc = os.confstr("CS_GNU_LIBC_VERSION")
        except (ValueError, OSError):
            glibc = None
        _LIBM["s"] = (bad == 0, bad, glibc)
    return _LIBM["s"]


def assert_parity(got, want, suite_tolerance=True):
    """MFCC f32 parity against the reference build's words: bit-exact when the host libm logf
    is the restated one; otherwise the reference suite's tolerance (MFCCF32.cpp:7-13:
    |err| <= 1e-5 + 1.2e-3 |ref|) is asserted and the test is SKIPPED as "libm differs" --
    a different libm, not a parity failure."""
    import pytest
    g = np.ascontiguousarray(got, np.float32)
    w = np.ascontiguousarray(want, np.float32)
    same = g.view(np.uint32) == w.view(np.uint32)
    ok, bad, glibc = host_libm_status()
    if ok:
        assert same.all(), (np.argwhere(~same)[:5], float(np.nanmax(np.abs(g - w))))
        return
    if suite_tolerance:
        assert np.all(np.abs(g - w) <= 1e-5 + 1.2e-3 * np.abs(w)), float(np.nanmax(np.abs(g - w)))
    pytest.skip(f"host libm differs ({glibc}: logf != restated glibc 2.35 __logf_fma on {bad} sampled inputs); "
                "suite tolerance checked, bit-exactness not assessable on this host")


def edge_filterbanks(n, rng):
    """Mel filter sets at the edges of the half spectrum (for the fixed-point back ends, which compute
    only the magnitudes some filter reads): bins 0 and fftLen/2, an empty filter, a narrow range that
    starts at an odd bin, the whole half spectrum.  Returns [(pos, len)] lists of uint32 arrays."""
    h = n // 2
    sets = [[(0, 3), (7, 0), (n // 4, min(40, h - n // 4)), (h - 9, 10)],
            [(n // 4 + 3, 5), (n // 4 + 5, 7)],
            [(h, 1), (0, 1)],
            [(0, h + 1)]]
    out = []
    for s in sets:
        out.append((np.array([p for p, _ in s], np.uint32), np.array([l for _, l in s], np.uint32)))
    return out
