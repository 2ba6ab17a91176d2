"""cmsisdsp_amd — Python face of the MI355X CMSIS-DSP backend (libcmsisdsp_mi355x.so).

Two layers, both thin over the C ABI (include/arm_math.h, include/arm_math_mi355x.h):

* drop-in, numpy in / numpy out, named and shaped like the reference's PythonWrapper
  (`cmsisdsp.arm_cfft_f32(inst, x, ifft, bitrev)` -> new array; PythonWrapper/cmsisdsp_pkg/
  src/cmsisdsp_transform.c:2074):  arm_cfft_f32 / _q31 / _q15, arm_rfft_fast_f32,
  arm_fir_f32 / _q15, arm_mat_mult_f32 with their *_init functions;
* batched, torch device tensors in place on a HIP stream: cfft_batch, rfft_fast_batch,
  fir_batch, mat_mult_batch.

The library is REQUIRED: importing works without a GPU, but every compute call goes to
the HIP kernels; there is no CPU fallback (a missing .so raises at import).
"""
import ctypes as C
import os

import numpy as np

from . import _abi
from ._abi import (arm_cfft_instance_f32, arm_cfft_instance_q15, arm_cfft_instance_q31,  # noqa: F401
                   arm_fir_instance_f32, arm_fir_instance_q15, arm_fir_instance_q31, arm_fir_instance_q7,
                   arm_matrix_instance_f32,
                   arm_rfft_fast_instance_f32, arm_mfcc_instance_f32, arm_mfcc_instance_q31, arm_mfcc_instance_q15,
                   arm_matrix_instance_q15, arm_matrix_instance_q7,
                   arm_matrix_instance_q31, arm_rfft_instance_q31, arm_rfft_instance_q15, ARM_MATH_SUCCESS,
                   ARM_MATH_ARGUMENT_ERROR, ARM_MATH_SIZE_MISMATCH)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CMSISDSP_MI355X_LIB",
                          os.path.join(os.path.dirname(_HERE), "lib", "libcmsisdsp_mi355x.so"))


def _load():
    # One HIP runtime per process: torch bundles its own libamdhip64 (SONAME
    # libamdhip64.so.7, same as ROCm's).  Loading torch first makes our library bind to
    # that already-loaded runtime instead of pulling in a second ROCr instance (two in
    # one process fail with "no ROCm-capable device").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"cmsisdsp_amd: native library missing at {LIB_PATH} "
                          f"(build it with `make -C cmsis-dsp_amd` or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    _abi.bind(lib, _abi.DROPIN)
    _abi.bind(lib, _abi.MFCC_LEN)
    _abi.bind(lib, _abi.RFFTQ_LEN)
    _abi.bind(lib, _abi.PARTIAL_FAST)
    _abi.bind(lib, _abi.BATCHED)
    return lib


lib = _load()


def version():
    return lib.arm_mi355x_version().decode()


def last_error():
    return lib.arm_mi355x_last_error(), lib.arm_mi355x_last_error_string().decode()


def _check_void(what):
    code, msg = last_error()
    if code:
        lib.arm_mi355x_clear_error()
        raise RuntimeError(f"{what}: device error {code}: {msg}")


def const_instance(name):
    """A pre-initialised const instance exported by the library (arm_const_structs.h)."""
    kind = {"f32": arm_cfft_instance_f32, "q31": arm_cfft_instance_q31, "q15": arm_cfft_instance_q15}
    if name.startswith("arm_rfft_fast_sR_f32"):
        return arm_rfft_fast_instance_f32.in_dll(lib, name)
    return kind[name.split("_")[3]].in_dll(lib, name)


# ------------------------------------------------------------------ drop-in (numpy)
def arm_cfft_init_f32(S, n):
    return lib.arm_cfft_init_f32(C.byref(S), n)


def arm_cfft_init_q31(S, n):
    return lib.arm_cfft_init_q31(C.byref(S), n)


def arm_cfft_init_q15(S, n):
    return lib.arm_cfft_init_q15(C.byref(S), n)


def _cfft(fn, dtype, S, x, ifft, bitrev):
    buf = np.ascontiguousarray(x, dtype=dtype).copy()
    fn(C.byref(S), buf.ctypes.data, ifft, bitrev)
    _check_void(fn.__name__)
    return buf


def arm_cfft_f32(S, x, ifftFlag, bitReverseFlag):
    return _cfft(lib.arm_cfft_f32, np.float32, S, x, ifftFlag, bitReverseFlag)


def arm_cfft_q31(S, x, ifftFlag, bitReverseFlag):
    return _cfft(lib.arm_cfft_q31, np.int32, S, x, ifftFlag, bitReverseFlag)


def arm_cfft_q15(S, x, ifftFlag, bitReverseFlag):
    return _cfft(lib.arm_cfft_q15, np.int16, S, x, ifftFlag, bitReverseFlag)


def arm_rfft_fast_init_f32(S, n):
    return lib.arm_rfft_fast_init_f32(C.byref(S), n)


def arm_rfft_fast_f32(S, x, ifftFlag):
    """Returns the output; like the reference, the forward transform also destroys the
    input buffer (here a private copy)."""
    p = np.ascontiguousarray(x, dtype=np.float32).copy()
    out = np.zeros(S.fftLenRFFT, dtype=np.float32)
    lib.arm_rfft_fast_f32(C.byref(S), p.ctypes.data, out.ctypes.data, ifftFlag)
    _check_void("arm_rfft_fast_f32")
    return out


def arm_rfft_init_q31(S, n, ifftFlagR, bitReverseFlag):
    return lib.arm_rfft_init_q31(C.byref(S), n, ifftFlagR, bitReverseFlag)


def arm_rfft_init_q15(S, n, ifftFlagR, bitReverseFlag):
    return lib.arm_rfft_init_q15(C.byref(S), n, ifftFlagR, bitReverseFlag)


def _rfft_fixed(kind, S, x):
    dt = np.int32 if kind == "q31" else np.int16
    src = np.ascontiguousarray(x, dtype=dt).copy()
    n = S.fftLenReal
    out = np.zeros(n if S.ifftFlagR == 1 else 2 * n, dtype=dt)
    fn = getattr(lib, f"arm_rfft_{kind}")
    fn(C.byref(S), src.ctypes.data, out.ctypes.data)
    _check_void(fn.__name__)
    return out


def arm_rfft_q31(S, x):
    """Forward: N samples -> 2N-word spectrum; inverse: spectrum (>= N+2 words) -> N samples
    (arm_rfft_q31.c:148-183; the input copy is consumed as in the reference)."""
    return _rfft_fixed("q31", S, x)


def arm_rfft_q15(S, x):
    return _rfft_fixed("q15", S, x)


def rfft_fixed_batch(S, src, dst, stream=None):
    """Batched arm_rfft_q31 / _q15 on device tensors: forward src [batch, N] (overwritten)
    -> dst [batch, 2N]; inverse src [batch, 2N] -> dst [batch, N]."""
    kind = "q31" if isinstance(S, arm_rfft_instance_q31) else "q15"
    fn = getattr(lib, f"arm_rfft_{kind}_batch")
    st = fn(C.byref(S), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), dst.shape[0], _stream_ptr(stream))
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")


class FirF32:
    """Streaming FIR f32 (arm_fir_init_f32 + arm_fir_f32): state carried across calls."""

    def __init__(self, coeffs, block_size):
        self.coeffs = np.ascontiguousarray(coeffs, dtype=np.float32)
        self.block_size = block_size
        self.state = np.zeros(len(self.coeffs) + block_size - 1, dtype=np.float32)
        self.S = arm_fir_instance_f32()
        lib.arm_fir_init_f32(C.byref(self.S), len(self.coeffs), self.coeffs.ctypes.data,
                             self.state.ctypes.data, block_size)

    def __call__(self, x):
        x = np.ascontiguousarray(x, dtype=np.float32)
        assert len(x) <= self.block_size
        y = np.empty_like(x)
        lib.arm_fir_f32(C.byref(self.S), x.ctypes.data, y.ctypes.data, len(x))
        _check_void("arm_fir_f32")
        return y


class FirQ15(FirF32):
    def __init__(self, coeffs, block_size):
        self.coeffs = np.ascontiguousarray(coeffs, dtype=np.int16)
        self.block_size = block_size
        self.state = np.zeros(len(self.coeffs) + block_size - 1, dtype=np.int16)
        self.S = arm_fir_instance_q15()
        lib.arm_fir_init_q15(C.byref(self.S), len(self.coeffs), self.coeffs.ctypes.data,
                             self.state.ctypes.data, block_size)

    def __call__(self, x):
        x = np.ascontiguousarray(x, dtype=np.int16)
        y = np.empty_like(x)
        lib.arm_fir_q15(C.byref(self.S), x.ctypes.data, y.ctypes.data, len(x))
        _check_void("arm_fir_q15")
        return y


class FirQ31(FirF32):
    """Streaming arm_fir_q31 (fast=False) or arm_fir_fast_q31 (fast=True)."""

    def __init__(self, coeffs, block_size, fast=False):
        self.coeffs = np.ascontiguousarray(coeffs, dtype=np.int32)
        self.block_size = block_size
        self.fn = lib.arm_fir_fast_q31 if fast else lib.arm_fir_q31
        self.state = np.zeros(len(self.coeffs) + block_size - 1, dtype=np.int32)
        self.S = arm_fir_instance_q31()
        lib.arm_fir_init_q31(C.byref(self.S), len(self.coeffs), self.coeffs.ctypes.data,
                             self.state.ctypes.data, block_size)

    def __call__(self, x):
        x = np.ascontiguousarray(x, dtype=np.int32)
        y = np.empty_like(x)
        self.fn(C.byref(self.S), x.ctypes.data, y.ctypes.data, len(x))
        _check_void(self.fn.__name__)
        return y


class FirQ7(FirF32):
    """Streaming arm_fir_q7."""

    def __init__(self, coeffs, block_size):
        self.coeffs = np.ascontiguousarray(coeffs, dtype=np.int8)
        self.block_size = block_size
        self.state = np.zeros(len(self.coeffs) + block_size - 1, dtype=np.int8)
        self.S = arm_fir_instance_q7()
        lib.arm_fir_init_q7(C.byref(self.S), len(self.coeffs), self.coeffs.ctypes.data,
                            self.state.ctypes.data, block_size)

    def __call__(self, x):
        x = np.ascontiguousarray(x, dtype=np.int8)
        y = np.empty_like(x)
        lib.arm_fir_q7(C.byref(self.S), x.ctypes.data, y.ctypes.data, len(x))
        _check_void("arm_fir_q7")
        return y


class FirFastQ15(FirQ15):
    """Streaming arm_fir_fast_q15."""

    def __call__(self, x):
        x = np.ascontiguousarray(x, dtype=np.int16)
        y = np.empty_like(x)
        lib.arm_fir_fast_q15(C.byref(self.S), x.ctypes.data, y.ctypes.data, len(x))
        _check_void("arm_fir_fast_q15")
        return y


def arm_mat_mult_f32(a, b):
    """(status, C) = A @ B through arm_mat_mult_f32 (row-major f32)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    c = np.zeros((a.shape[0], b.shape[1]), dtype=np.float32)
    A, B, Cm = arm_matrix_instance_f32(), arm_matrix_instance_f32(), arm_matrix_instance_f32()
    lib.arm_mat_init_f32(C.byref(A), a.shape[0], a.shape[1], a.ctypes.data)
    lib.arm_mat_init_f32(C.byref(B), b.shape[0], b.shape[1], b.ctypes.data)
    lib.arm_mat_init_f32(C.byref(Cm), c.shape[0], c.shape[1], c.ctypes.data)
    st = lib.arm_mat_mult_f32(C.byref(A), C.byref(B), C.byref(Cm))
    _check_void("arm_mat_mult_f32")
    return st, c


class MfccF32:
    """arm_mfcc_init_f32 + arm_mfcc_f32 with the instance's tables kept alive.
    dct: [nbDctOutputs, nbMelFilters]; pos/lengths: per Mel filter; coefs: concatenated
    filter weights; window: fftLen.  Tables may be numpy arrays (host) or torch device
    tensors (their data_ptr is used)."""

    def __init__(self, fft_len, dct, pos, lengths, coefs, window):
        def keep(a, dt):
            if hasattr(a, "data_ptr"):
                return a, a.data_ptr()
            a = np.ascontiguousarray(a, dtype=dt)
            return a, a.ctypes.data
        self._t = [keep(dct, np.float32), keep(pos, np.uint32), keep(lengths, np.uint32), keep(coefs, np.float32),
                   keep(window, np.float32)]
        self.nb_mel = int(len(lengths))
        self.nb_dct = int(dct.shape[0])
        self.fft_len = int(fft_len)
        self.S = arm_mfcc_instance_f32()
        st = lib.arm_mfcc_init_f32(C.byref(self.S), self.fft_len, self.nb_mel, self.nb_dct,
                                   *[p for _, p in self._t])
        if st != ARM_MATH_SUCCESS:
            raise ValueError(f"arm_mfcc_init_f32({fft_len}) -> {st}")

    def __call__(self, x):
        """One frame (numpy) -> nbDctOutputs coefficients (the reference's call shape)."""
        src = np.ascontiguousarray(x, dtype=np.float32).copy()
        dst = np.zeros(self.nb_dct, dtype=np.float32)
        tmp = np.zeros(2 * self.fft_len, dtype=np.float32)
        lib.arm_mfcc_f32(C.byref(self.S), src.ctypes.data, dst.ctypes.data, tmp.ctypes.data)
        _check_void("arm_mfcc_f32")
        return dst

    def batch(self, frames, out=None, work=None, stream=None):
        """frames: torch device tensor [batch, fftLen] (overwritten) -> [batch, nbDct]."""
        import torch
        b = frames.shape[0]
        out = torch.empty((b, self.nb_dct), dtype=torch.float32, device=frames.device) if out is None else out
        work = torch.empty_like(frames) if work is None else work
        st = lib.arm_mfcc_f32_batch(C.byref(self.S), C.c_void_p(frames.data_ptr()), C.c_void_p(out.data_ptr()),
                                    C.c_void_p(work.data_ptr()), b, _stream_ptr(stream))
        if st != ARM_MATH_SUCCESS:
            raise RuntimeError(f"arm_mfcc_f32_batch -> {st}: {last_error()[1]}")
        return out


class _MfccFixed:
    """arm_mfcc_init_<t> + arm_mfcc_<t> (bit-exact) with the instance's tables kept alive.
    dct: [nbDctOutputs, nbMelFilters]; pos/lengths: per Mel filter; coefs: concatenated filter
    weights; window: fftLen.  Tables: numpy (host) or torch device tensors."""
    T = None            # "q31" | "q15"

    def __init__(self, fft_len, dct, pos, lengths, coefs, window):
        dt = np.int32 if self.T == "q31" else np.int16

        def keep(a, d):
            if hasattr(a, "data_ptr"):
                return a, a.data_ptr()
            a = np.ascontiguousarray(a, dtype=d)
            return a, a.ctypes.data
        self._dt = dt
        self._t = [keep(dct, dt), keep(pos, np.uint32), keep(lengths, np.uint32), keep(coefs, dt), keep(window, dt)]
        self.nb_mel = int(len(lengths))
        self.nb_dct = int(dct.shape[0])
        self.fft_len = int(fft_len)
        self.S = (arm_mfcc_instance_q31 if self.T == "q31" else arm_mfcc_instance_q15)()
        st = getattr(lib, f"arm_mfcc_init_{self.T}")(C.byref(self.S), self.fft_len, self.nb_mel, self.nb_dct,
                                                     *[p for _, p in self._t])
        if st != ARM_MATH_SUCCESS:
            raise ValueError(f"arm_mfcc_init_{self.T}({fft_len}) -> {st}")

    def __call__(self, x):
        """One frame (numpy) -> nbDctOutputs coefficients (the reference's call shape)."""
        src = np.ascontiguousarray(x, dtype=self._dt).copy()
        dst = np.zeros(self.nb_dct, dtype=self._dt)
        tmp = np.zeros(2 * self.fft_len, dtype=np.int32)
        st = getattr(lib, f"arm_mfcc_{self.T}")(C.byref(self.S), src.ctypes.data, dst.ctypes.data, tmp.ctypes.data)
        if st != ARM_MATH_SUCCESS:
            raise RuntimeError(f"arm_mfcc_{self.T} -> {st}: {last_error()[1]}")
        return dst

    def batch(self, frames, out=None, work=None, stream=None):
        """frames: torch device tensor [batch, fftLen] (int32 / int16, overwritten) -> [batch, nbDct]."""
        import torch
        b = frames.shape[0]
        out = torch.empty((b, self.nb_dct), dtype=frames.dtype, device=frames.device) if out is None else out
        work = torch.empty((b, 2 * self.fft_len), dtype=frames.dtype, device=frames.device) if work is None else work
        st = getattr(lib, f"arm_mfcc_{self.T}_batch")(C.byref(self.S), C.c_void_p(frames.data_ptr()),
                                                      C.c_void_p(out.data_ptr()), C.c_void_p(work.data_ptr()), b,
                                                      _stream_ptr(stream))
        if st != ARM_MATH_SUCCESS:
            raise RuntimeError(f"arm_mfcc_{self.T}_batch -> {st}: {last_error()[1]}")
        return out


class MfccQ31(_MfccFixed):
    """arm_mfcc_q31: q31 frames -> q8.23 coefficients."""
    T = "q31"


class MfccQ15(_MfccFixed):
    """arm_mfcc_q15: q15 frames -> q8.7 coefficients."""
    T = "q15"


# ------------------------------------------------------------------ batched (torch, device)
def _stream_ptr(stream):
    if stream is None:
        import torch
        stream = torch.cuda.current_stream()
    return C.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))


_CFFT_BATCH = {"f32": ("arm_cfft_f32_batch", 2), "q31": ("arm_cfft_q31_batch", 2),
               "q15": ("arm_cfft_q15_batch", 2)}


def cfft_batch(S, data, ifft, bitrev, stream=None, kind=None):
    """In-place CFFT of every row of `data` (torch device tensor [batch, 2*N])."""
    if kind is None:
        kind = {arm_cfft_instance_f32: "f32", arm_cfft_instance_q31: "q31",
                arm_cfft_instance_q15: "q15"}[type(S)]
    fn = getattr(lib, _CFFT_BATCH[kind][0])
    batch = data.numel() // (2 * S.fftLen)
    st = fn(C.byref(S), C.c_void_p(data.data_ptr()), batch, ifft, bitrev, _stream_ptr(stream))
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")


def cfft_batch_multi(S, shards, ifft, bitrev, kind=None):
    """In-place CFFT of every row of every tensor in `shards` (torch tensors [batch_s, 2*N],
    each on its own device) through one arm_cfft_*_batch_multi call (synchronous)."""
    if kind is None:
        kind = {arm_cfft_instance_f32: "f32", arm_cfft_instance_q31: "q31",
                arm_cfft_instance_q15: "q15"}[type(S)]
    k = len(shards)
    # the C side runs each shard on the library's own stream of that device: order it after
    # whatever torch work is still producing the shards
    import torch
    for d in sorted({t.device.index for t in shards}):
        torch.cuda.synchronize(d)
    devs = (C.c_int * k)(*[t.device.index for t in shards])
    ptrs = (C.c_void_p * k)(*[t.data_ptr() for t in shards])
    cnts = (C.c_uint32 * k)(*[t.numel() // (2 * S.fftLen) for t in shards])
    fn = getattr(lib, f"arm_cfft_{kind}_batch_multi")
    st = fn(C.byref(S), k, devs, ptrs, cnts, ifft, bitrev)
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")


def device_count():
    return lib.arm_mi355x_device_count()


def table_cache_bytes():
    """Device bytes held by the content-keyed cache of host tables / coefficients."""
    return lib.arm_mi355x_table_cache_bytes()


def set_table_cache_limit(nbytes):
    lib.arm_mi355x_set_table_cache_limit(C.c_size_t(nbytes))


def release_thread_resources():
    """Free the calling thread's drop-in streams, scratch and staging now (automatic at the exit
    of any thread but the main one)."""
    lib.arm_mi355x_release_thread_resources()


def thread_resource_owners():
    """Number of threads currently holding per-thread runtime resources."""
    return lib.arm_mi355x_thread_resource_owners()


RFFT_P_SCRATCH = 1     # ARM_MI355X_RFFT_P_SCRATCH


def rfft_fast_batch(S, p, out, ifft, stream=None, p_scratch=False):
    """Batched arm_rfft_fast_f32; p_scratch=True: arm_rfft_fast_f32_batch_ex with
    ARM_MI355X_RFFT_P_SCRATCH (p is scratch, the forward skips writing the inner CFFT back)."""
    batch = p.numel() // S.fftLenRFFT
    if p_scratch:
        st = lib.arm_rfft_fast_f32_batch_ex(C.byref(S), C.c_void_p(p.data_ptr()), C.c_void_p(out.data_ptr()),
                                            batch, ifft, RFFT_P_SCRATCH, _stream_ptr(stream))
    else:
        st = lib.arm_rfft_fast_f32_batch(C.byref(S), C.c_void_p(p.data_ptr()), C.c_void_p(out.data_ptr()), batch,
                                         ifft, _stream_ptr(stream))
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"arm_rfft_fast_f32_batch -> {st}: {last_error()[1]}")


_FIR_BATCH = {"f32": "arm_fir_f32_batch", "f32_fma": "arm_fir_f32_batch_fma", "q15": "arm_fir_q15_batch",
              "q31": "arm_fir_q31_batch",
              "fast_q15": "arm_fir_fast_q15_batch", "fast_q31": "arm_fir_fast_q31_batch", "q7": "arm_fir_q7_batch"}


def fir_batch(S, src, dst, hist, stream=None, q15=False, kind=None):
    """src/dst: [batch, blockSize] device tensors; hist: [batch, numTaps-1] device state.
    kind: f32 | f32_fma (opt-in tolerance path) | q15 | q31 | fast_q15 | fast_q31 | q7 (default from
    the instance type / q15 flag)."""
    if kind is None:
        kind = "q15" if q15 else {arm_fir_instance_f32: "f32", arm_fir_instance_q15: "q15",
                                  arm_fir_instance_q31: "q31", arm_fir_instance_q7: "q7"}[type(S)]
    batch, block = src.shape
    fn = getattr(lib, _FIR_BATCH[kind])
    st = fn(C.byref(S), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), block, batch,
            C.c_void_p(hist.data_ptr() if hist is not None and hist.numel() else 0), _stream_ptr(stream))
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")


def fir_batch_multi(S, shards, kind=None):
    """FIR over filter shards on several devices through one arm_fir_*_batch_multi call
    (synchronous): shards = [(src, dst, hist), ...], torch tensors [batch_s, blockSize] /
    [batch_s, numTaps-1] on each shard's device."""
    import torch
    if kind is None:
        kind = {arm_fir_instance_f32: "f32", arm_fir_instance_q15: "q15",
                arm_fir_instance_q31: "q31", arm_fir_instance_q7: "q7"}[type(S)]
    k = len(shards)
    for d in sorted({t[0].device.index for t in shards}):
        torch.cuda.synchronize(d)
    block = shards[0][0].shape[1] if k else 0
    devs = (C.c_int * k)(*[t[0].device.index for t in shards])
    src = (C.c_void_p * k)(*[t[0].data_ptr() for t in shards])
    dst = (C.c_void_p * k)(*[t[1].data_ptr() for t in shards])
    hist = (C.c_void_p * k)(*[t[2].data_ptr() if t[2] is not None and t[2].numel() else 0 for t in shards])
    cnts = (C.c_uint32 * k)(*[t[0].shape[0] for t in shards])
    fn = getattr(lib, f"arm_fir_{kind}_batch_multi")
    st = fn(C.byref(S), k, devs, src, dst, hist, block, cnts)
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")


def mat_mult_batch_multi(shards):
    """c[i] = a[i] @ b[i] per shard through one arm_mat_mult_*_batch_multi call (synchronous):
    shards = [(a, b, c), ...] with [batch_s, M, K] x [batch_s, K, N] -> [batch_s, M, N] tensors
    on each shard's device (f32 / int16 / int32)."""
    import torch
    a0, b0, _ = shards[0]
    m, k_, n = a0.shape[1], a0.shape[2], b0.shape[2]
    kind, inst = {torch.float32: ("f32", arm_matrix_instance_f32), torch.int16: ("q15", arm_matrix_instance_q15),
                  torch.int32: ("q31", arm_matrix_instance_q31), torch.int8: ("q7", arm_matrix_instance_q7)}[a0.dtype]
    for d in sorted({t[0].device.index for t in shards}):
        torch.cuda.synchronize(d)
    k = len(shards)
    A, B, Cm = inst(m, k_, None), inst(k_, n, None), inst(m, n, None)
    devs = (C.c_int * k)(*[t[0].device.index for t in shards])
    pa, pb, pc = ((C.c_void_p * k)(*[t[i].data_ptr() for t in shards]) for i in range(3))
    cnts = (C.c_uint32 * k)(*[t[0].shape[0] for t in shards])
    fn = getattr(lib, f"arm_mat_mult_{kind}_batch_multi")
    st = fn(C.byref(A), C.byref(B), C.byref(Cm), k, devs, pa, pb, pc, cnts)
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")


def arm_conv(kind, a, b):
    """arm_conv_f32 / _q15 / _q31 / _q7 (drop-in, numpy): len(a) + len(b) - 1 samples."""
    dt = {"f32": np.float32, "q15": np.int16, "q31": np.int32, "q7": np.int8}[kind]
    a = np.ascontiguousarray(a, dtype=dt)
    b = np.ascontiguousarray(b, dtype=dt)
    y = np.zeros(len(a) + len(b) - 1, dtype=dt)
    getattr(lib, f"arm_conv_{kind}")(a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data)
    _check_void(f"arm_conv_{kind}")
    return y


def conv_batch(a, b, out, stream=None):
    """out[i] = a[i] (*) b[i]; a [batch, La], b [batch, Lb] or [Lb] (shared), out [batch, La+Lb-1]."""
    import torch
    kind = {torch.float32: "f32", torch.int16: "q15", torch.int32: "q31", torch.int8: "q7"}[a.dtype]
    batch, la = a.shape
    lb = b.shape[-1]
    sb = 0 if b.dim() == 1 else b.stride(0)
    fn = getattr(lib, f"arm_conv_{kind}_batch")
    st = fn(C.c_void_p(a.data_ptr()), la, a.stride(0), C.c_void_p(b.data_ptr()), lb, sb,
            C.c_void_p(out.data_ptr()), batch, _stream_ptr(stream))
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")


def arm_conv_family(fn, a, b, first=0, num=0, fill=0):
    """Drop-in (numpy) call of arm_<fn>, fn in _abi.CONV_FULL + _abi.CONV_PARTIAL (e.g.
    "correlate_q15", "conv_partial_f32", "conv_fast_q31"): returns (pDst, status); pDst is
    pre-filled with `fill`, since partial / correlate leave the words they do not compute."""
    dt = {"f32": np.float32, "q15": np.int16, "q31": np.int32, "q7": np.int8}[fn.split("_")[-1]]
    a = np.ascontiguousarray(a, dtype=dt)
    b = np.ascontiguousarray(b, dtype=dt)
    n = 2 * max(len(a), len(b)) - 1 if fn.startswith("correlate") else len(a) + len(b) - 1
    y = np.full(n, fill, dtype=dt)
    f = getattr(lib, f"arm_{fn}")
    if fn.startswith("conv_partial"):
        st = f(a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data, first, num)
    else:
        f(a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data)
        st = ARM_MATH_SUCCESS
    _check_void(f"arm_{fn}")
    return y, st


def conv_family_batch(fn, a, b, out, first=0, num=0, stream=None):
    """arm_<fn>_batch on torch device tensors: a [batch, La], b [batch, Lb] or [Lb] (shared),
    out [batch, La+Lb-1] (conv), [batch, 2*max-1] (correlate) or [batch, num] (partial)."""
    batch, la = a.shape
    lb = b.shape[-1]
    sb = 0 if b.dim() == 1 else b.stride(0)
    fn_ = getattr(lib, f"arm_{fn}_batch")
    args = [C.c_void_p(a.data_ptr()), la, a.stride(0), C.c_void_p(b.data_ptr()), lb, sb, C.c_void_p(out.data_ptr())]
    if fn.startswith("conv_partial"):
        args += [first, num]
    st = fn_(*args, batch, _stream_ptr(stream))
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"arm_{fn}_batch -> {st}: {last_error()[1]}")


def arm_mat_mult_fixed(kind, a, b):
    """(status, C) = A @ B through arm_mat_mult_q7 / _q15 / _q31 / _fast_q15 / _fast_q31 (kind
    "q7", "q15", "q31", "opt_q31", "fast_q15", "fast_q31"; row-major)."""
    base = "q7" if kind == "q7" else kind[-3:]
    dt = {"q7": np.int8, "q15": np.int16, "q31": np.int32}[base]
    inst = {"q7": arm_matrix_instance_q7, "q15": arm_matrix_instance_q15, "q31": arm_matrix_instance_q31}[base]
    a = np.ascontiguousarray(a, dtype=dt)
    b = np.ascontiguousarray(b, dtype=dt)
    c = np.zeros((a.shape[0], b.shape[1]), dtype=dt)
    A, B, Cm = inst(), inst(), inst()
    init = getattr(lib, f"arm_mat_init_{base}")
    init(C.byref(A), a.shape[0], a.shape[1], a.ctypes.data)
    init(C.byref(B), b.shape[0], b.shape[1], b.ctypes.data)
    init(C.byref(Cm), c.shape[0], c.shape[1], c.ctypes.data)
    fn = getattr(lib, f"arm_mat_mult_{kind}")
    st = fn(C.byref(A), C.byref(B), C.byref(Cm), None) if base in ("q15", "q7") or kind == "opt_q31" else \
        fn(C.byref(A), C.byref(B), C.byref(Cm))
    _check_void(f"arm_mat_mult_{kind}")
    return st, c


def mat_mult_batch(a, b, c, stream=None, fast=False):
    """c[i] = a[i] @ b[i] for device tensors [batch, M, K] x [batch, K, N] -> [batch, M, N];
    float32 -> arm_mat_mult_f32_batch, int8 -> _q7, int16 -> _q15, int32 -> _q31 (fast=True:
    _fast_q15 / _fast_q31)."""
    import torch
    batch, m, k = a.shape
    n = b.shape[2]
    kind, inst, ptr = {torch.float32: ("f32", arm_matrix_instance_f32, _abi.c_f32p),
                       torch.int16: ("q15", arm_matrix_instance_q15, _abi.c_i16p),
                       torch.int32: ("q31", arm_matrix_instance_q31, _abi.c_i32p),
                       torch.int8: ("q7", arm_matrix_instance_q7, _abi.c_i8p)}[a.dtype]
    A, B, Cm = inst(m, k, C.cast(a.data_ptr(), ptr)), inst(k, n, C.cast(b.data_ptr(), ptr)), \
        inst(m, n, C.cast(c.data_ptr(), ptr))
    fn = getattr(lib, f"arm_mat_mult_{'fast_' if fast and kind != 'f32' else ''}{kind}_batch")
    st = fn(C.byref(A), C.byref(B), C.byref(Cm), batch, _stream_ptr(stream))
    if st != ARM_MATH_SUCCESS:
        raise RuntimeError(f"{fn.__name__} -> {st}: {last_error()[1]}")