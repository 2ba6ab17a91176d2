"""The reference test framework's acceptance checks (Testing/FrameworkSource/Error.cpp:515-705,
Testing/FrameworkInclude/Error.h:165-179), restated for numpy."""
import numpy as np


def snr_db(ref, out):
    """ASSERT_SNR: 10*log10(sum ref^2 / sum (ref-out)^2), computed in double."""
    ref = np.asarray(ref, dtype=np.float64)
    err = ref - np.asarray(out, dtype=np.float64)
    e = np.sum(err * err)
    return np.inf if e == 0 else 10.0 * np.log10(np.sum(ref * ref) / e)


def close_error(out, ref, abs_err, rel_err):
    """ASSERT_CLOSE_ERROR: |out - ref| <= abs + rel*|ref| elementwise."""
    out = np.asarray(out, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return bool(np.all(np.abs(out - ref) <= abs_err + rel_err * np.abs(ref)))


def rel_error(out, ref, rel_err):
    """ASSERT_REL_ERROR: |out - ref| <= rel*|ref| (where ref != 0)."""
    out = np.asarray(out, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    nz = ref != 0
    return bool(np.all(np.abs(out[nz] - ref[nz]) <= rel_err * np.abs(ref[nz])))


def near_eq(out, ref, abs_err):
    """ASSERT_NEAR_EQ on integer words."""
    return int(np.max(np.abs(np.asarray(out, np.int64) - np.asarray(ref, np.int64)))) <= abs_err


# Per-suite thresholds of the reference tests (Testing/Source/Tests/*.cpp)
CFFT_TOL = {"f32": dict(snr=120, abs=8e-5, rel=2e-5),     # TransformCF32.cpp:6-8
            "q31": dict(snr=90, abs=53),                   # TransformCQ31.cpp:6-7
            "q15": dict(snr=30, abs=15)}                   # TransformCQ15.cpp:6-7
FIR_TOL = {"f32": dict(snr=120, rel=3e-5),                 # FIRF32.cpp:5,11
           "q15": dict(snr=59, abs=2)}                     # FIRQ15.cpp:5-7
MAT_TOL = dict(snr=120, abs=1e-5, rel=1e-6)                # BinaryTestsF32.cpp:5,13-17
