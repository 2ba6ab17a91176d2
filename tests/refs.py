"""Test-side access to the two CPU checkers (test infrastructure only — never the product):

* `ref_lib()`    — oracle/_ref/libcmsisdsp_ref.so: the reference's own scalar C, compiled
                   from /root/reference by oracle/ref.mk (travels to the GPU box prebuilt);
* `oracle_lib()` — oracle/_build/liboracle.so: our plain-C restatement (oracle/src/*.c),
                   exported with an `oracle_` prefix and the same C ABI.

Both are wrapped by `Host`, a numpy in / numpy out driver with the reference's call
shapes, so a test reads `host.cfft("f32", n, x, ifft, bitrev)` for either checker.
"""
import ctypes as C
import os

import numpy as np

from cmsisdsp_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libcmsisdsp_ref.so")
# CMSISDSP_ORACLE_SO overrides the restatement (tools/oracle_san.sh: the ASan/UBSan build)
ORACLE_SO = os.environ.get("CMSISDSP_ORACLE_SO") or os.path.join(ROOT, "oracle", "_build", "liboracle.so")

_INST = {"f32": _abi.arm_cfft_instance_f32, "q31": _abi.arm_cfft_instance_q31, "q15": _abi.arm_cfft_instance_q15}
DTYPE = {"f32": np.float32, "q31": np.int32, "q15": np.int16, "q7": np.int8}


class Host:
    def __init__(self, lib, prefix):
        self.lib, self.p = lib, prefix
        _abi.bind(lib, _abi.DROPIN, prefix)

    def fn(self, name):
        return getattr(self.lib, self.p + name)

    def cfft_instance(self, kind, n):
        S = _INST[kind]()
        st = self.fn(f"arm_cfft_init_{kind}")(C.byref(S), n)
        assert st == 0, (kind, n, st)
        return S

    def cfft(self, kind, n, x, ifft, bitrev):
        S = self.cfft_instance(kind, n)
        buf = np.ascontiguousarray(x, dtype=DTYPE[kind]).copy()
        assert buf.size == 2 * n
        self.fn(f"arm_cfft_{kind}")(C.byref(S), buf.ctypes.data, ifft, bitrev)
        return buf

    def cfft_many(self, kind, n, x, ifft, bitrev):
        """x: [batch, 2n] -> per-row transforms (a Python loop over the scalar call)."""
        S = self.cfft_instance(kind, n)
        out = np.ascontiguousarray(x, dtype=DTYPE[kind]).copy()
        f = self.fn(f"arm_cfft_{kind}")
        for r in range(out.shape[0]):
            f(C.byref(S), out[r].ctypes.data, ifft, bitrev)
        return out

    def rfft(self, n, x, ifft):
        S = _abi.arm_rfft_fast_instance_f32()
        assert self.fn("arm_rfft_fast_init_f32")(C.byref(S), n) == 0
        p = np.ascontiguousarray(x, dtype=np.float32).copy()
        out = np.zeros(n, dtype=np.float32)
        self.fn("arm_rfft_fast_f32")(C.byref(S), p.ctypes.data, out.ctypes.data, ifft)
        return out, p

    def rfft_fixed(self, kind, n, x, ifft, bitrev=1):
        """arm_rfft_q31 / _q15 on one signal: forward x = N words -> (2N-word spectrum, the
        overwritten input); inverse x = spectrum (>= N+2 words) -> (N words, x)."""
        inst = _abi.arm_rfft_instance_q31 if kind == "q31" else _abi.arm_rfft_instance_q15
        dt = DTYPE[kind]
        S = inst()
        st = self.fn(f"arm_rfft_init_{kind}")(C.byref(S), n, ifft, bitrev)
        assert st == 0, (kind, n, st)
        src = np.ascontiguousarray(x, dtype=dt).copy()
        out = np.zeros(2 * n if ifft != 1 else n, dtype=dt)
        self.fn(f"arm_rfft_{kind}")(C.byref(S), src.ctypes.data, out.ctypes.data)
        return out, src

    def mfcc(self, cfg, frames):
        """cfg: dict with fftLen, dct [nbDct x nbMel], pos, len, coefs, window; frames:
        [batch, fftLen] -> [batch, nbDct] (one arm_mfcc_f32 call per frame, zeroed pTmp)."""
        n = int(cfg["fftLen"])
        keep = [np.ascontiguousarray(cfg["dct"], dtype=np.float32), np.ascontiguousarray(cfg["pos"], dtype=np.uint32),
                np.ascontiguousarray(cfg["len"], dtype=np.uint32), np.ascontiguousarray(cfg["coefs"], dtype=np.float32),
                np.ascontiguousarray(cfg["window"], dtype=np.float32)]
        nb_mel, nb_dct = keep[1].size, keep[0].shape[0]
        S = _abi.arm_mfcc_instance_f32()
        st = self.fn("arm_mfcc_init_f32")(C.byref(S), n, nb_mel, nb_dct, *[k.ctypes.data for k in keep])
        assert st == 0, st
        frames = np.atleast_2d(np.asarray(frames, dtype=np.float32))
        out = np.zeros((frames.shape[0], nb_dct), dtype=np.float32)
        f = self.fn("arm_mfcc_f32")
        for r in range(frames.shape[0]):
            src = frames[r].copy()
            tmp = np.zeros(2 * n, dtype=np.float32)
            f(C.byref(S), src.ctypes.data, out[r].ctypes.data, tmp.ctypes.data)
        return out

    def mfcc_q15(self, cfg, frames):
        """arm_mfcc_q15 per frame (q15 tables and frames, q31 pTmp of 2*fftLen words)."""
        n = int(cfg["fftLen"])
        keep = [np.ascontiguousarray(cfg["dct"], dtype=np.int16), np.ascontiguousarray(cfg["pos"], dtype=np.uint32),
                np.ascontiguousarray(cfg["len"], dtype=np.uint32), np.ascontiguousarray(cfg["coefs"], dtype=np.int16),
                np.ascontiguousarray(cfg["window"], dtype=np.int16)]
        nb_mel, nb_dct = keep[1].size, keep[0].shape[0]
        S = _abi.arm_mfcc_instance_q15()
        st = self.fn("arm_mfcc_init_q15")(C.byref(S), n, nb_mel, nb_dct, *[k.ctypes.data for k in keep])
        assert st == 0, st
        frames = np.atleast_2d(np.asarray(frames, dtype=np.int16))
        out = np.zeros((frames.shape[0], nb_dct), dtype=np.int16)
        f = self.fn("arm_mfcc_q15")
        for r in range(frames.shape[0]):
            src = frames[r].copy()
            tmp = np.zeros(2 * n, dtype=np.int32)
            f(C.byref(S), src.ctypes.data, out[r].ctypes.data, tmp.ctypes.data)
        return out

    def mfcc_q31(self, cfg, frames):
        """cfg: dict with fftLen, dct [nbDct x nbMel] q31, pos, len, coefs q31, window q31;
        frames: [batch, fftLen] int32 -> [batch, nbDct] int32 (one arm_mfcc_q31 call per
        frame on a copy, zeroed pTmp of 2*fftLen words)."""
        n = int(cfg["fftLen"])
        keep = [np.ascontiguousarray(cfg["dct"], dtype=np.int32), np.ascontiguousarray(cfg["pos"], dtype=np.uint32),
                np.ascontiguousarray(cfg["len"], dtype=np.uint32), np.ascontiguousarray(cfg["coefs"], dtype=np.int32),
                np.ascontiguousarray(cfg["window"], dtype=np.int32)]
        nb_mel, nb_dct = keep[1].size, keep[0].shape[0]
        S = _abi.arm_mfcc_instance_q31()
        st = self.fn("arm_mfcc_init_q31")(C.byref(S), n, nb_mel, nb_dct, *[k.ctypes.data for k in keep])
        assert st == 0, st
        frames = np.atleast_2d(np.asarray(frames, dtype=np.int32))
        out = np.zeros((frames.shape[0], nb_dct), dtype=np.int32)
        f = self.fn("arm_mfcc_q31")
        for r in range(frames.shape[0]):
            src = frames[r].copy()
            tmp = np.zeros(2 * n, dtype=np.int32)
            f(C.byref(S), src.ctypes.data, out[r].ctypes.data, tmp.ctypes.data)
        return out

    def fir(self, kind, coeffs, blocks):
        """Stream `blocks` (list of 1-D arrays, each <= the block size) through one filter;
        returns (outputs, final state buffer).  kind: f32, q15, q31, fast_q15, fast_q31."""
        base = kind.split("_")[-1]
        dt = DTYPE[base]
        inst = {"f32": _abi.arm_fir_instance_f32, "q15": _abi.arm_fir_instance_q15,
                "q31": _abi.arm_fir_instance_q31, "q7": _abi.arm_fir_instance_q7}[base]()
        c = np.ascontiguousarray(coeffs, dtype=dt)
        bs = max(len(b) for b in blocks)
        state = np.zeros(len(c) + bs - 1, dtype=dt)
        self.fn(f"arm_fir_init_{base}")(C.byref(inst), len(c), c.ctypes.data, state.ctypes.data, bs)
        outs = []
        for b in blocks:
            b = np.ascontiguousarray(b, dtype=dt)
            y = np.zeros_like(b)
            self.fn(f"arm_fir_{kind}")(C.byref(inst), b.ctypes.data, y.ctypes.data, len(b))
            outs.append(y)
        self._keep = (c, state)
        return outs, state.copy()

    def multirate(self, fn, factor, coeffs, blocks, block_size=None):
        """Stream `blocks` through one arm_fir_decimate_* / arm_fir_interpolate_* instance
        (fn e.g. "decimate_fast_q15", "interpolate_f32"; factor = M or L): returns
        (init status, outputs, final state buffer)."""
        base = fn.split("_")[-1]
        dt = DTYPE[base]
        decim = fn.startswith("decimate")
        c = np.ascontiguousarray(coeffs, dtype=dt)
        bs = block_size or max(len(b) for b in blocks)
        if decim:
            inst = _abi.arm_fir_decimate_instance()
            state = np.zeros(len(c) + bs - 1, dtype=dt)
            st = self.fn(f"arm_fir_decimate_init_{base}")(C.byref(inst), len(c), factor, c.ctypes.data,
                                                            state.ctypes.data, bs)
        else:
            inst = _abi.arm_fir_interpolate_instance()
            state = np.zeros(bs + max(len(c) // max(factor, 1), 1) - 1, dtype=dt)
            st = self.fn(f"arm_fir_interpolate_init_{base}")(C.byref(inst), factor, len(c), c.ctypes.data,
                                                               state.ctypes.data, bs)
        if st != 0:
            return st, [], state
        outs = []
        f = self.fn(f"arm_fir_{fn}")
        for b in blocks:
            b = np.ascontiguousarray(b, dtype=dt)
            y = np.zeros(len(b) // factor if decim else len(b) * factor, dtype=dt)
            f(C.byref(inst), b.ctypes.data, y.ctypes.data, len(b))
            outs.append(y)
        self._keep = (c, state)
        return st, outs, state.copy()

    def lattice(self, kind, coeffs, blocks, state_mem=None):
        """Stream `blocks` through one arm_fir_lattice_<kind> instance: returns (outputs,
        final state).  state_mem(n, dtype) may supply the state buffer as (pointer, reader)."""
        dt = DTYPE[kind]
        c = np.ascontiguousarray(coeffs, dtype=dt)
        inst = _abi.arm_fir_lattice_instance()
        if state_mem is None:
            state = np.full(len(c), 5, dtype=dt)                  # init must zero it
            sptr, sread = state.ctypes.data, state.copy
        else:
            sptr, sread = state_mem(len(c), dt)
        self.fn(f"arm_fir_lattice_init_{kind}")(C.byref(inst), len(c), c.ctypes.data, sptr)
        f = self.fn(f"arm_fir_lattice_{kind}")
        outs = []
        for b in blocks:
            b = np.ascontiguousarray(b, dtype=dt)
            y = np.zeros(len(b), dtype=dt)
            f(C.byref(inst), b.ctypes.data, y.ctypes.data, len(b))
            outs.append(y)
        self._keep = (c,)
        return outs, sread()

    def sparse(self, kind, coeffs, delays, max_delay, blocks, block_size=None, state_mem=None):
        """Stream `blocks` through one arm_fir_sparse_<kind> instance: returns (outputs, final
        circular state, final stateIndex).  state_mem(n, dtype) may supply the state buffer
        (e.g. device memory) as (pointer, reader)."""
        dt = DTYPE[kind]
        c = np.ascontiguousarray(coeffs, dtype=dt)
        d = np.ascontiguousarray(delays, dtype=np.int32)
        bs = block_size or max(len(b) for b in blocks)
        inst = _abi.arm_fir_sparse_instance()
        if state_mem is None:
            state = np.full(max_delay + bs, 7, dtype=dt)       # init must zero it
            sptr, sread = state.ctypes.data, state.copy
        else:
            sptr, sread = state_mem(max_delay + bs, dt)
        self.fn(f"arm_fir_sparse_init_{kind}")(C.byref(inst), len(c), c.ctypes.data, sptr, d.ctypes.data,
                                                max_delay, bs)
        f = self.fn(f"arm_fir_sparse_{kind}")
        outs = []
        for b in blocks:
            b = np.ascontiguousarray(b, dtype=dt)
            y = np.zeros(len(b), dtype=dt)
            sin = np.zeros(len(b), dtype=dt)
            if kind in ("q15", "q7"):
                sout = np.zeros(len(b), dtype=np.int32)
                f(C.byref(inst), b.ctypes.data, y.ctypes.data, sin.ctypes.data, sout.ctypes.data, len(b))
            else:
                f(C.byref(inst), b.ctypes.data, y.ctypes.data, sin.ctypes.data, len(b))
            outs.append(y)
        self._keep = (c, d)
        return outs, sread(), inst.stateIndex

    def conv(self, kind, a, b):
        dt = DTYPE[kind]
        a = np.ascontiguousarray(a, dtype=dt)
        b = np.ascontiguousarray(b, dtype=dt)
        y = np.zeros(len(a) + len(b) - 1, dtype=dt)
        self.fn(f"arm_conv_{kind}")(a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data)
        return y

    def conv_family(self, fn, a, b, first=0, num=0, fill=0):
        """arm_<fn> for fn in _abi.CONV_FULL + CONV_PARTIAL on one pair: returns (pDst, status)
        with pDst pre-filled with `fill` (partial / correlate leave words untouched)."""
        dt = DTYPE[fn.split("_")[-1]]
        a = np.ascontiguousarray(a, dtype=dt)
        b = np.ascontiguousarray(b, dtype=dt)
        n = 2 * max(len(a), len(b)) - 1 if fn.startswith("correlate") else len(a) + len(b) - 1
        y = np.full(n, fill, dtype=dt)
        f = self.fn(f"arm_{fn}")
        if fn.startswith("conv_partial"):
            return y, f(a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data, first, num)
        f(a.ctypes.data, len(a), b.ctypes.data, len(b), y.ctypes.data)
        return y, 0

    def mat_mult_fixed(self, kind, a, b):
        """arm_mat_mult_q7 / _q15 / _q31 / _opt_q31 / _fast_q15 / _fast_q31: returns (status, C)."""
        base = kind[-3:] if kind != "q7" else "q7"
        dt = {"q7": np.int8, "q15": np.int16, "q31": np.int32}[base]
        inst = {"q7": _abi.arm_matrix_instance_q7, "q15": _abi.arm_matrix_instance_q15,
                "q31": _abi.arm_matrix_instance_q31}[base]
        a = np.ascontiguousarray(a, dtype=dt)
        b = np.ascontiguousarray(b, dtype=dt)
        c = np.zeros((a.shape[0], b.shape[1]), dtype=dt)
        A, B, Cm = inst(), inst(), inst()
        init = self.fn(f"arm_mat_init_{base}")
        init(C.byref(A), a.shape[0], a.shape[1], a.ctypes.data)
        init(C.byref(B), b.shape[0], b.shape[1], b.ctypes.data)
        init(C.byref(Cm), c.shape[0], c.shape[1], c.ctypes.data)
        if base in ("q15", "q7") or kind == "opt_q31":
            state = np.zeros(a.shape[1] * b.shape[1] + 16, dtype=dt)
            st = self.fn(f"arm_mat_mult_{kind}")(C.byref(A), C.byref(B), C.byref(Cm), state.ctypes.data)
        else:
            st = self.fn(f"arm_mat_mult_{kind}")(C.byref(A), C.byref(B), C.byref(Cm))
        return st, c

    def mat_mult_fmaf(self, a, b):
        """oracle_mat_mult_f32_fmaf (restatement only): the product's stated k-ordered fmaf-chain
        semantics for arm_mat_mult_f32 -> (status, C)."""
        a = np.ascontiguousarray(a, dtype=np.float32)
        b = np.ascontiguousarray(b, dtype=np.float32)
        c = np.zeros((a.shape[0], b.shape[1]), dtype=np.float32)
        A, B, Cm = (_abi.arm_matrix_instance_f32() for _ in range(3))
        init = self.fn("arm_mat_init_f32")
        init(C.byref(A), a.shape[0], a.shape[1], a.ctypes.data)
        init(C.byref(B), b.shape[0], b.shape[1], b.ctypes.data)
        init(C.byref(Cm), c.shape[0], c.shape[1], c.ctypes.data)
        f = self.lib.oracle_mat_mult_f32_fmaf
        f.restype = C.c_int
        f.argtypes = [C.c_void_p] * 3
        st = f(C.byref(A), C.byref(B), C.byref(Cm))
        return st, c

    def mat_mult(self, a, b):
        a = np.ascontiguousarray(a, dtype=np.float32)
        b = np.ascontiguousarray(b, dtype=np.float32)
        c = np.zeros((a.shape[0], b.shape[1]), dtype=np.float32)
        A, B, Cm = (_abi.arm_matrix_instance_f32() for _ in range(3))
        init = self.fn("arm_mat_init_f32")
        init(C.byref(A), a.shape[0], a.shape[1], a.ctypes.data)
        init(C.byref(B), b.shape[0], b.shape[1], b.ctypes.data)
        init(C.byref(Cm), c.shape[0], c.shape[1], c.ctypes.data)
        st = self.fn("arm_mat_mult_f32")(C.byref(A), C.byref(B), C.byref(Cm))
        return st, c


_cache = {}


def ref_lib():
    if "ref" not in _cache:
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(f"{REF_SO} missing: build it with `make -f oracle/ref.mk` (needs /root/reference)")
        _cache["ref"] = Host(C.CDLL(REF_SO), "")
    return _cache["ref"]


def oracle_lib():
    if "oracle" not in _cache:
        if not os.path.exists(ORACLE_SO):
            raise FileNotFoundError(f"{ORACLE_SO} missing: build it with `make -C oracle`")
        _cache["oracle"] = Host(C.CDLL(ORACLE_SO), "oracle_")
    return _cache["oracle"]


# ------------------------------------------------------------------ seeded inputs
def splitmix64(seed, n):
    """The SplitMix64 stream (Steele et al.); bench.py and tests share it for inputs."""
    out = np.empty(n, dtype=np.uint64)
    s = np.uint64(seed)
    with np.errstate(over="ignore"):
        for i in range(n):
            s = s + np.uint64(0x9E3779B97F4A7C15)
            z = s
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            out[i] = z ^ (z >> np.uint64(31))
    return out


def rand_input(kind, n_words, seed, dist="uniform"):
    rng = np.random.default_rng(seed)
    if kind == "f32":
        if dist == "uniform":
            return rng.uniform(-1.0, 1.0, n_words).astype(np.float32)
        if dist == "large":
            return (rng.standard_normal(n_words) * 1e4).astype(np.float32)
        raise ValueError(dist)
    info = np.iinfo(DTYPE[kind])
    if dist == "uniform":           # full range: exercises wrap / saturation
        return rng.integers(info.min, info.max, n_words, endpoint=True, dtype=np.int64).astype(DTYPE[kind])
    if dist == "sine":              # reference-style noisy sine, cmsisdsp/fixedpoint.py round+saturate
        t = np.arange(n_words // 2)
        v = 0.7 * np.sin(2 * np.pi * 13 * t / max(1, n_words // 2)) + 0.05 * rng.standard_normal(n_words // 2)
        z = np.empty(n_words)
        z[0::2] = v
        z[1::2] = 0.05 * rng.standard_normal(n_words // 2)
        scale = 2.0 ** (31 if kind == "q31" else 15)
        return np.clip(np.round(z * scale), info.min, info.max).astype(DTYPE[kind])
    if dist == "extreme":           # all min / max words
        return rng.choice(np.array([info.min, info.max, 0, -1], dtype=DTYPE[kind]), n_words)
    raise ValueError(dist)
