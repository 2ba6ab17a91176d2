"""`cmsisdsp`-compatible Python module over the MI355X library.

Same function names, argument order and return conventions as the reference's CPython
extension (PythonWrapper/cmsisdsp_pkg/src/cmsisdsp_transform.c, _filtering.c, _matrix.c,
as exercised by PythonWrapper/examples/testdsp*.py, testrfft_all.py, testmfcc.py) for the
functions this backend provides: numpy (or list) in, a new numpy array out, instances as
opaque objects.  Every call runs on the GPU through libcmsisdsp_mi355x.so (the drop-in C
ABI, host buffers staged through device memory); there is no CPU implementation here.

    import sys; sys.path.insert(0, "cmsis-dsp_amd")
    import cmsisdsp as dsp
    S = dsp.arm_cfft_instance_f32(); dsp.arm_cfft_init_f32(S, 1024)
    y = dsp.arm_cfft_f32(S, x, 0, 1)
"""
import ctypes as _C

import numpy as _np

import cmsisdsp_amd as _amd
from cmsisdsp_amd import _abi
from . import datatype  # noqa: F401

_lib = _amd.lib
_ARCH_DEFAULT = 1                      # ARM_MATH_DEFAULT_TARGET_ARCH = ARM_MATH_SCALAR_ARCH (arm_math_types.h)


def has_neon():
    return False


# ------------------------------------------------------------------ instances
class _Instance:
    _struct = None

    def __init__(self):
        self._s = self._struct()
        self._keep = []

    def __getattr__(self, name):            # accessor methods: inst.fftLen(), inst.numTaps() ...
        s = object.__getattribute__(self, "_s")
        if any(f == name for f, _ in s._fields_):
            return lambda: getattr(s, name)
        raise AttributeError(name)


def _make(name, struct):
    return type(name, (_Instance,), {"_struct": struct})


arm_cfft_instance_f32 = _make("arm_cfft_instance_f32", _abi.arm_cfft_instance_f32)
arm_cfft_instance_q31 = _make("arm_cfft_instance_q31", _abi.arm_cfft_instance_q31)
arm_cfft_instance_q15 = _make("arm_cfft_instance_q15", _abi.arm_cfft_instance_q15)
arm_rfft_fast_instance_f32 = _make("arm_rfft_fast_instance_f32", _abi.arm_rfft_fast_instance_f32)
arm_fir_instance_f32 = _make("arm_fir_instance_f32", _abi.arm_fir_instance_f32)
arm_fir_instance_q31 = _make("arm_fir_instance_q31", _abi.arm_fir_instance_q31)
arm_fir_instance_q15 = _make("arm_fir_instance_q15", _abi.arm_fir_instance_q15)
arm_fir_instance_q7 = _make("arm_fir_instance_q7", _abi.arm_fir_instance_q7)
arm_mfcc_instance_f32 = _make("arm_mfcc_instance_f32", _abi.arm_mfcc_instance_f32)
arm_mfcc_instance_q31 = _make("arm_mfcc_instance_q31", _abi.arm_mfcc_instance_q31)
arm_mfcc_instance_q15 = _make("arm_mfcc_instance_q15", _abi.arm_mfcc_instance_q15)
for _t in ("f32", "q31", "q15"):
    globals()[f"arm_fir_decimate_instance_{_t}"] = _make(f"arm_fir_decimate_instance_{_t}",
                                                         _abi.arm_fir_decimate_instance)
    globals()[f"arm_fir_interpolate_instance_{_t}"] = _make(f"arm_fir_interpolate_instance_{_t}",
                                                            _abi.arm_fir_interpolate_instance)
for _t in ("f32", "q31", "q15"):
    globals()[f"arm_fir_lattice_instance_{_t}"] = _make(f"arm_fir_lattice_instance_{_t}", _abi.arm_fir_lattice_instance)
for _t in ("f32", "q31", "q15", "q7"):
    globals()[f"arm_fir_sparse_instance_{_t}"] = _make(f"arm_fir_sparse_instance_{_t}", _abi.arm_fir_sparse_instance)
del _t
arm_rfft_instance_q31 = _make("arm_rfft_instance_q31", _abi.arm_rfft_instance_q31)
arm_rfft_instance_q15 = _make("arm_rfft_instance_q15", _abi.arm_rfft_instance_q15)

_DT = {"f32": _np.float32, "q31": _np.int32, "q15": _np.int16, "q7": _np.int8}


def _arr(x, dt):
    return _np.ascontiguousarray(_np.asarray(x).astype(dt, copy=False))


def _check(what):
    code, msg = _amd.last_error()
    if code:
        _lib.arm_mi355x_clear_error()
        raise RuntimeError(f"{what}: device error {code}: {msg}")


# ------------------------------------------------------------------ complex FFT
def _cfft_init(kind):
    def init(inst, fftLen):
        return getattr(_lib, f"arm_cfft_init_{kind}")(_C.byref(inst._s), int(fftLen))
    init.__name__ = f"arm_cfft_init_{kind}"
    return init


def _cfft(kind):
    def run(inst, p1, ifftFlag, bitReverseFlag=1, tmp=None):
        buf = _arr(p1, _DT[kind]).copy()
        getattr(_lib, f"arm_cfft_{kind}")(_C.byref(inst._s), buf.ctypes.data, int(ifftFlag), int(bitReverseFlag))
        _check(f"arm_cfft_{kind}")
        return buf
    run.__name__ = f"arm_cfft_{kind}"
    return run


arm_cfft_init_f32, arm_cfft_init_q31, arm_cfft_init_q15 = (_cfft_init(k) for k in ("f32", "q31", "q15"))
arm_cfft_f32, arm_cfft_q31, arm_cfft_q15 = (_cfft(k) for k in ("f32", "q31", "q15"))


def arm_cfft_tmp_buffer_size(dt, nbSamples, buf_id, arch=None):
    return 0                                  # no user temporary: work space lives on the device


def arm_cfft_output_buffer_size(dt, nbSamples, arch=None):
    return 2 * int(nbSamples)


def arm_cifft_output_buffer_size(dt, nbSamples, arch=None):
    """cmsisdsp_transform.c cmsis_arm_cifft_output_buffer_size ("II|$I", :3032-3050), answered
    by the library's arm_cifft_output_buffer_size (arm_transform_buffer_sizes.c)."""
    return int(_lib.arm_cifft_output_buffer_size(_ARCH_DEFAULT if arch is None else int(arch), int(dt),
                                                 int(nbSamples)))


# ------------------------------------------------------------------ real FFT (fast)
def arm_rfft_fast_init_f32(inst, fftLen):
    return _lib.arm_rfft_fast_init_f32(_C.byref(inst._s), int(fftLen))


def arm_rfft_fast_f32(inst, p, ifftFlag, tmp=None):
    src = _arr(p, _np.float32).copy()
    out = _np.zeros(inst._s.fftLenRFFT, dtype=_np.float32)
    _lib.arm_rfft_fast_f32(_C.byref(inst._s), src.ctypes.data, out.ctypes.data, int(ifftFlag))
    _check("arm_rfft_fast_f32")
    return out


# ------------------------------------------------------------------ real FFT, q31 / q15
# cmsisdsp_transform.c:2275-2313 (init: "Oi|ii"), :2180-2273 / :2317-2405 (rfft: "OO|i$O",
# the ifft / tmp arguments exist for the Neon API only): output fftLenReal words for an
# inverse instance, 2*fftLenReal otherwise; the input is converted (copied) first.
def _rfft_q_init(kind):
    def init(inst, fftLenReal, ifftFlagR=0, bitReverseFlag=0):
        return getattr(_lib, f"arm_rfft_init_{kind}")(_C.byref(inst._s), int(fftLenReal), int(ifftFlagR),
                                                      int(bitReverseFlag))
    init.__name__ = f"arm_rfft_init_{kind}"
    return init


def _rfft_q(kind):
    def rfft(inst, pSrc, ifft=0, tmp=None):
        s = inst._s
        n = int(s.fftLenReal)
        src = _np.zeros(2 * n, dtype=_DT[kind])           # room for the widest read (inverse: N+2)
        x = _arr(pSrc, _DT[kind]).ravel()
        src[:min(x.size, 2 * n)] = x[:2 * n]
        out = _np.zeros(2 * n, dtype=_DT[kind])
        getattr(_lib, f"arm_rfft_{kind}")(_C.byref(s), src.ctypes.data, out.ctypes.data)
        _check(f"arm_rfft_{kind}")
        return out[:n] if s.ifftFlagR else out
    rfft.__name__ = f"arm_rfft_{kind}"
    return rfft


arm_rfft_init_q31 = _rfft_q_init("q31")
arm_rfft_init_q15 = _rfft_q_init("q15")
arm_rfft_q31 = _rfft_q("q31")
arm_rfft_q15 = _rfft_q("q15")


def arm_rfft_tmp_buffer_size(dt, nbSamples, buf_id, arch=None):
    return 0


def arm_rfft_output_buffer_size(dt, nbSamples, arch=None):
    """arm_transform_buffer_sizes.c:204-230 (generic arch): float N, fixed point 2N."""
    from . import datatype as _dt
    return 2 * int(nbSamples) if dt in (_dt.Q31, _dt.Q15) else int(nbSamples)


def arm_rifft_input_buffer_size(dt, nbSamples, arch=None):
    """arm_transform_buffer_sizes.c:245-263: float N, fixed point N + 2."""
    from . import datatype as _dt
    return int(nbSamples) + 2 if dt in (_dt.Q31, _dt.Q15) else int(nbSamples)


# ------------------------------------------------------------------ FIR
def _fir_init(kind):
    def init(inst, numTaps, pCoeffs, pState):
        c = _arr(pCoeffs, _DT[kind])
        state = _arr(pState, _DT[kind]).copy()
        block = max(1, len(state) - int(numTaps) + 1)
        inst._keep = [c, state]
        inst._block = block
        getattr(_lib, f"arm_fir_init_{kind}")(_C.byref(inst._s), int(numTaps), c.ctypes.data, state.ctypes.data, block)
        _check(f"arm_fir_init_{kind}")
        return 0
    init.__name__ = f"arm_fir_init_{kind}"
    return init


def _fir(name, kind):
    def run(inst, pSrc):
        x = _arr(pSrc, _DT[kind])
        if len(x) > inst._block:
            raise ValueError(f"{name}: {len(x)} samples > the blockSize the state was sized for ({inst._block})")
        y = _np.zeros_like(x)
        getattr(_lib, name)(_C.byref(inst._s), x.ctypes.data, y.ctypes.data, len(x))
        _check(name)
        return y
    run.__name__ = name
    return run


arm_fir_init_f32, arm_fir_init_q31, arm_fir_init_q15, arm_fir_init_q7 = (_fir_init(k) for k in ("f32", "q31", "q15", "q7"))
arm_fir_q7 = _fir("arm_fir_q7", "q7")
arm_fir_f32 = _fir("arm_fir_f32", "f32")
arm_fir_q31 = _fir("arm_fir_q31", "q31")
arm_fir_q15 = _fir("arm_fir_q15", "q15")
arm_fir_fast_q31 = _fir("arm_fir_fast_q31", "q31")
arm_fir_fast_q15 = _fir("arm_fir_fast_q15", "q15")


# ------------------------------------------------------------------ multirate FIR
# cmsisdsp_filtering.c cmsis_arm_fir_decimate_init_* ("OhiOO": blockSize = len(pState) -
# len(pCoeffs) + 1, :4742-4772) / cmsis_arm_fir_interpolate_init_* ("OihOO", same blockSize
# rule, :5164-5190) return the status; cmsis_arm_fir_decimate_* returns len(pSrc) / M words,
# cmsis_arm_fir_interpolate_* len(pSrc) * L words (:4706-4740, :5128-5160).
def _mr_init(family, kind):
    name = f"arm_fir_{family}_init_{kind}"

    def init(inst, a, b, pCoeffs, pState):
        c = _arr(pCoeffs, _DT[kind])
        state = _arr(pState, _DT[kind]).copy()
        block = len(state) - len(c) + 1
        inst._keep = [c, state]
        st = getattr(_lib, name)(_C.byref(inst._s), int(a), int(b), c.ctypes.data, state.ctypes.data, block)
        _check(name)
        return st
    init.__name__ = name
    return init


def _mr(family, fn, kind):
    name = f"arm_fir_{fn}"

    def run(inst, pSrc):
        x = _arr(pSrc, _DT[kind])
        n = len(x) // inst._s.M if family == "decimate" else len(x) * inst._s.L
        y = _np.zeros(n, dtype=_DT[kind])
        getattr(_lib, name)(_C.byref(inst._s), x.ctypes.data, y.ctypes.data, len(x))
        _check(name)
        return y
    run.__name__ = name
    return run


for _k in ("f32", "q31", "q15"):
    globals()[f"arm_fir_decimate_init_{_k}"] = _mr_init("decimate", _k)
    globals()[f"arm_fir_interpolate_init_{_k}"] = _mr_init("interpolate", _k)
    globals()[f"arm_fir_decimate_{_k}"] = _mr("decimate", f"decimate_{_k}", _k)
    globals()[f"arm_fir_interpolate_{_k}"] = _mr("interpolate", f"interpolate_{_k}", _k)
arm_fir_decimate_fast_q15 = _mr("decimate", "decimate_fast_q15", "q15")
arm_fir_decimate_fast_q31 = _mr("decimate", "decimate_fast_q31", "q31")
del _k


# cmsisdsp_filtering.c cmsis_arm_fir_lattice_init_* ("OhOO": S, numStages, pCoeffs, pState) and
# cmsis_arm_fir_lattice_* ("OO": S, pSrc; returns len(pSrc) words).
def _lattice_init(kind):
    name = f"arm_fir_lattice_init_{kind}"

    def init(inst, numStages, pCoeffs, pState):
        c = _arr(pCoeffs, _DT[kind])
        state = _np.zeros(max(len(_np.asarray(pState)), int(numStages)), dtype=_DT[kind])
        inst._keep = [c, state]
        getattr(_lib, name)(_C.byref(inst._s), int(numStages), c.ctypes.data, state.ctypes.data)
        _check(name)
    init.__name__ = name
    return init


def _lattice(kind):
    name = f"arm_fir_lattice_{kind}"

    def run(inst, pSrc):
        x = _arr(pSrc, _DT[kind])
        y = _np.zeros(len(x), dtype=_DT[kind])
        getattr(_lib, name)(_C.byref(inst._s), x.ctypes.data, y.ctypes.data, len(x))
        _check(name)
        return y
    run.__name__ = name
    return run


for _k in ("f32", "q31", "q15"):
    globals()[f"arm_fir_lattice_init_{_k}"] = _lattice_init(_k)
    globals()[f"arm_fir_lattice_{_k}"] = _lattice(_k)
del _k


# cmsisdsp_filtering.c cmsis_arm_fir_sparse_init_* ("OhOOOh": S, numTaps, pCoeffs, pState,
# pTapDelay, maxDelay; blockSize = len(pState) - len(pCoeffs) + 1, :6666-6690) and
# cmsis_arm_fir_sparse_f32 ("OOO": S, pSrc, pScratchIn; returns len(pSrc) words, :6628-6662).
# The module keeps its own state copy of at least maxDelay + blockSize words and refuses a
# block that would not fit it (the C call would run past the caller's state).
def _sparse_init(kind):
    name = f"arm_fir_sparse_init_{kind}"

    def init(inst, numTaps, pCoeffs, pState, pTapDelay, maxDelay):
        c = _arr(pCoeffs, _DT[kind])
        d = _arr(pTapDelay, _np.int32)
        block = max(len(_np.asarray(pState)) - len(c) + 1, 0)
        state = _np.zeros(max(len(_np.asarray(pState)), int(maxDelay) + block), dtype=_DT[kind])
        inst._keep = [c, d, state]
        getattr(_lib, name)(_C.byref(inst._s), int(numTaps), c.ctypes.data, state.ctypes.data, d.ctypes.data,
                            int(maxDelay), block)
        _check(name)
    init.__name__ = name
    return init


def _sparse(kind):
    name = f"arm_fir_sparse_{kind}"

    def run(inst, pSrc, pScratchIn=None, pScratchOut=None):
        x = _arr(pSrc, _DT[kind])
        if inst._s.maxDelay + len(x) > len(inst._keep[2]):
            raise ValueError(f"{name}: maxDelay + len(pSrc) exceeds the state given to the init call")
        y = _np.zeros(len(x), dtype=_DT[kind])
        if kind in ("q15", "q7"):
            getattr(_lib, name)(_C.byref(inst._s), x.ctypes.data, y.ctypes.data, None, None, len(x))
        else:
            getattr(_lib, name)(_C.byref(inst._s), x.ctypes.data, y.ctypes.data, None, len(x))
        _check(name)
        return y
    run.__name__ = name
    return run


for _k in ("f32", "q31", "q15", "q7"):
    globals()[f"arm_fir_sparse_init_{_k}"] = _sparse_init(_k)
    globals()[f"arm_fir_sparse_{_k}"] = _sparse(_k)
del _k


# ------------------------------------------------------------------ matrix multiply
def arm_mat_mult_f32(pSrcA, pSrcB):
    """(status, A @ B) as in the reference binding."""
    return _amd.arm_mat_mult_f32(_arr(pSrcA, _np.float32), _arr(pSrcB, _np.float32))


def arm_mat_mult_q31(pSrcA, pSrcB):
    return _amd.arm_mat_mult_fixed("q31", _arr(pSrcA, _np.int32), _arr(pSrcB, _np.int32))


def arm_mat_mult_opt_q31(pSrcA, pSrcB, pState=None):
    """cmsisdsp_matrix.c cmsis_arm_mat_mult_opt_q31 ("OOO" -> (status, C), :1302-1330)."""
    return _amd.arm_mat_mult_fixed("opt_q31", _arr(pSrcA, _np.int32), _arr(pSrcB, _np.int32))


def arm_mat_mult_q7(pSrcA, pSrcB, pState=None):
    """cmsisdsp_matrix.c cmsis_arm_mat_mult_q7 ("OOO" -> (status, C), :1110-1140)."""
    return _amd.arm_mat_mult_fixed("q7", _arr(pSrcA, _np.int8), _arr(pSrcB, _np.int8))


def arm_mat_mult_q15(pSrcA, pSrcB, pState=None):
    return _amd.arm_mat_mult_fixed("q15", _arr(pSrcA, _np.int16), _arr(pSrcB, _np.int16))


def arm_mat_mult_fast_q31(pSrcA, pSrcB):
    """cmsisdsp_matrix.c cmsis_arm_mat_mult_fast_q31: (status, C)."""
    return _amd.arm_mat_mult_fixed("fast_q31", _arr(pSrcA, _np.int32), _arr(pSrcB, _np.int32))


def arm_mat_mult_fast_q15(pSrcA, pSrcB, pState=None):
    return _amd.arm_mat_mult_fixed("fast_q15", _arr(pSrcA, _np.int16), _arr(pSrcB, _np.int16))


# ------------------------------------------------------------------ convolution
def _conv(kind, dt):
    def run(pSrcA, srcALen, pSrcB, srcBLen):
        """Full linear convolution, srcALen + srcBLen - 1 samples (reference binding
        PythonWrapper/cmsisdsp_pkg/src/cmsisdsp_filtering.c cmsis_arm_conv_*)."""
        a = _arr(pSrcA, dt)[:int(srcALen)]
        b = _arr(pSrcB, dt)[:int(srcBLen)]
        return _amd.arm_conv(kind, a, b)
    run.__name__ = f"arm_conv_{kind}"
    return run


arm_conv_f32 = _conv("f32", _np.float32)
arm_conv_q15 = _conv("q15", _np.int16)
arm_conv_q31 = _conv("q31", _np.int32)
arm_conv_q7 = _conv("q7", _np.int8)


# cmsisdsp_filtering.c cmsis_arm_conv_fast_* ("OiOi", srcALen + srcBLen - 1 words),
# cmsis_arm_correlate_* ("OiOi", 2 * max(srcALen, srcBLen) - 1 words, :6244-6276) and
# cmsis_arm_conv_partial_* ("OiOiii" -> (status, srcALen + srcBLen - 1 words), :4313-4350).
# The binding's output buffer is uninitialised where the C function does not write; here
# those words are zero.
def _conv_family(fn):
    dt = _DT[fn.split("_")[-1]]

    def run(pSrcA, srcALen, pSrcB, srcBLen, *partial):
        a = _arr(pSrcA, dt)[:int(srcALen)]
        b = _arr(pSrcB, dt)[:int(srcBLen)]
        y, st = _amd.arm_conv_family(fn, a, b, *[int(v) for v in partial])
        return (st, y) if partial else y
    run.__name__ = f"arm_{fn}"
    return run


for _fn in ("conv_fast_q15", "conv_fast_q31", "correlate_f32", "correlate_q15", "correlate_q31", "correlate_fast_q15",
            "correlate_fast_q31", "conv_partial_f32", "conv_partial_q15", "conv_partial_q31", "conv_partial_fast_q15",
            "conv_partial_fast_q31", "correlate_q7", "conv_partial_q7"):
    globals()[f"arm_{_fn}"] = _conv_family(_fn)
del _fn


# The scratch-buffer ("_opt") forms, cmsisdsp_filtering.c cmsis_arm_conv_opt_q15 / _q7 /
# _fast_opt_q15 ("OiOiOO", :3993, :4231, :4112), cmsis_arm_correlate_opt_q15 / _fast_opt_q15
# ("OiOiO", :6316, :6431), cmsis_arm_correlate_opt_q7 ("OiOiOO", :6546) -> the output words;
# cmsis_arm_conv_partial_opt_q15 / _q7 / _fast_opt_q15 ("OiOiiiOO", :4354, :4616, :4485) ->
# (status, srcALen + srcBLen - 1 words).  The caller's scratch arrays are accepted and not
# touched: the C call gets scratch of its own, sized as the reference requires
# (pScratch1 srcALen + 2 srcBLen - 2 q15 words, pScratch2 min(srcALen, srcBLen)).
def _conv_opt(fn):
    dt = _DT[fn.split("_")[-1]]
    n_scratch = _abi.CONV_OPT_FULL.get(fn, 2)

    def run(pSrcA, srcALen, pSrcB, srcBLen, *rest):
        a = _arr(pSrcA, dt)[:int(srcALen)]
        b = _arr(pSrcB, dt)[:int(srcBLen)]
        s1 = _np.zeros(len(a) + 2 * len(b) + 16, _np.int16)
        s2 = _np.zeros(len(a) + 2 * len(b) + 16, _np.int16)
        f = getattr(_lib, f"arm_{fn}")
        if fn in _abi.CONV_OPT_PARTIAL:
            first, num = int(rest[0]), int(rest[1])
            y = _np.zeros(len(a) + len(b) - 1, dt)
            st = f(a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data, first, num, s1.ctypes.data,
                   s2.ctypes.data)
            _check(f"arm_{fn}")
            return st, y
        n = 2 * max(len(a), len(b)) - 1 if fn.startswith("correlate") else len(a) + len(b) - 1
        y = _np.zeros(n, dt)
        args = [a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data, s1.ctypes.data]
        if n_scratch == 2:
            args.append(s2.ctypes.data)
        f(*args)
        _check(f"arm_{fn}")
        return y
    run.__name__ = f"arm_{fn}"
    return run


for _fn in (*_abi.CONV_OPT_FULL, *_abi.CONV_OPT_PARTIAL):
    globals()[f"arm_{_fn}"] = _conv_opt(_fn)
del _fn


# ------------------------------------------------------------------ MFCC
def arm_mfcc_init_f32(inst, fftLen, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths,
                      filterCoefs, windowCoefs):
    keep = [_arr(dctCoefs, _np.float32).reshape(-1), _arr(filterPos, _np.uint32), _arr(filterLengths, _np.uint32),
            _arr(filterCoefs, _np.float32), _arr(windowCoefs, _np.float32)]
    inst._keep = keep
    return _lib.arm_mfcc_init_f32(_C.byref(inst._s), int(fftLen), int(nbMelFilters), int(nbDctOutputs),
                                  *[k.ctypes.data for k in keep])


def arm_mfcc_f32(inst, pSrc, pTmp, tmp2=None):
    src = _arr(pSrc, _np.float32).copy()
    out = _np.zeros(inst._s.nbDctOutputs, dtype=_np.float32)
    tmp = _np.zeros(2 * inst._s.fftLen, dtype=_np.float32)
    _lib.arm_mfcc_f32(_C.byref(inst._s), src.ctypes.data, out.ctypes.data, tmp.ctypes.data)
    _check("arm_mfcc_f32")
    return out


def _mfcc_fixed_init(t, dt):
    def init(inst, fftLen, nbMelFilters, nbDctOutputs, dctCoefs, filterPos, filterLengths, filterCoefs, windowCoefs):
        keep = [_arr(dctCoefs, dt).reshape(-1), _arr(filterPos, _np.uint32), _arr(filterLengths, _np.uint32),
                _arr(filterCoefs, dt), _arr(windowCoefs, dt)]
        inst._keep = keep
        return getattr(_lib, f"arm_mfcc_init_{t}")(_C.byref(inst._s), int(fftLen), int(nbMelFilters),
                                                   int(nbDctOutputs), *[k.ctypes.data for k in keep])
    init.__name__ = f"arm_mfcc_init_{t}"
    return init


def _mfcc_fixed(t, dt):
    # cmsisdsp_transform.c:2821-2870 (q15), the q31 analogue: returns (status, pDst)
    def mfcc(inst, pSrc, pTmp, tmp2=None):
        src = _arr(pSrc, dt).copy()
        out = _np.zeros(inst._s.nbDctOutputs, dtype=dt)
        tmp = _np.zeros(2 * inst._s.fftLen, dtype=_np.int32)
        st = getattr(_lib, f"arm_mfcc_{t}")(_C.byref(inst._s), src.ctypes.data, out.ctypes.data, tmp.ctypes.data)
        return st, out
    mfcc.__name__ = f"arm_mfcc_{t}"
    return mfcc


arm_mfcc_init_q31 = _mfcc_fixed_init("q31", _np.int32)
arm_mfcc_init_q15 = _mfcc_fixed_init("q15", _np.int16)
arm_mfcc_q31 = _mfcc_fixed("q31", _np.int32)
arm_mfcc_q15 = _mfcc_fixed("q15", _np.int16)


def arm_mfcc_tmp_buffer_size(dt, fftLen, buf_id, arch=None, use_cfft=0):
    return 2 * int(fftLen) if buf_id == 1 else 0
