"""Sparse FIR: arm_fir_sparse_{f32,q31,q15,q7} (+ inits and the batched device API).

CPU: the oracle restatement (oracle/src/oracle_multirate.c) equals the reference build
(oracle/_ref, Source/FilteringFunctions/arm_fir_sparse_*.c, arm_fir_sparse_init_*.c) bit for
bit: outputs of consecutive calls, the final circular state buffer and stateIndex, over tap
counts, delay sets (0, maxDelay, repeated, unsorted), block sizes hitting the unrolled and
remainder loops, block sizes that shrink between calls (the circular length changes with
blockSize), full-range and all-minimum fixed-point words (wrap / saturation).
GPU: the product (drop-in through host and device buffers; the batched device API over
several streams and two calls each, histories carried in d_hist) equals the reference build.
(numTaps == 1 is not compared: the reference's numTaps - 2 loop counter underflows.)
"""
import ctypes as C

import numpy as np
import pytest

import refs
from cmsisdsp_amd import _abi

KINDS = ["f32", "q31", "q15", "q7"]
# (numTaps, maxDelay, block sizes)
CASES = [(2, 0, [16, 16]), (5, 7, [8, 8, 8]), (16, 100, [64, 64, 20]), (33, 1000, [4096, 4096]),
         (3, 5, [1, 1, 1, 1, 1, 1, 1, 1]), (64, 300, [257, 257]), (10, 65, [3, 5, 2])]


def data(kind, n, rng, dist="full"):
    if kind == "f32":
        return rng.standard_normal(n).astype(np.float32)
    info = np.iinfo(refs.DTYPE[kind])
    if dist == "min":
        return np.full(n, info.min, refs.DTYPE[kind])
    return rng.integers(info.min, info.max, n, endpoint=True).astype(refs.DTYPE[kind])


def case(kind, taps, max_delay, blocks, seed, dist="full"):
    rng = np.random.default_rng(seed)
    c = data(kind, taps, rng, dist)
    if kind == "f32":
        c = (c / np.sqrt(taps)).astype(np.float32)
    d = rng.integers(0, max_delay, taps, endpoint=True).astype(np.int32)
    d[0] = max_delay
    if taps > 2:
        d[1] = 0
        d[2] = d[0]                                  # a repeated delay
    return c, d, [data(kind, b, rng, dist) for b in blocks]


def same(a, b):
    ya, sa, ia = a
    yb, sb, ib = b
    assert len(ya) == len(yb)
    for k, (u, v) in enumerate(zip(ya, yb)):
        assert u.tobytes() == v.tobytes(), k
    assert sa.tobytes() == sb.tobytes()
    assert ia == ib


# ------------------------------------------------------------------ CPU: oracle == reference
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("taps,max_delay,blocks", CASES)
def test_sparse_oracle_equals_reference(oracle, ref, kind, taps, max_delay, blocks):
    c, d, xs = case(kind, taps, max_delay, blocks, taps * 11 + max_delay)
    same(oracle.sparse(kind, c, d, max_delay, xs), ref.sparse(kind, c, d, max_delay, xs))


@pytest.mark.parametrize("kind", ["q31", "q15", "q7"])
def test_sparse_extreme_words(oracle, ref, kind):
    """All-minimum samples and taps: the q31 sums wrap, the outputs saturate."""
    c, d, xs = case(kind, 40, 50, [64, 64], 3, dist="min")
    same(oracle.sparse(kind, c, d, 50, xs), ref.sparse(kind, c, d, 50, xs))


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module")
def product(dsp):
    return refs.Host(dsp.lib, "")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_sparse_dropin_bitexact(product, torch_gpu, ref, kind):
    for taps, max_delay, blocks in CASES:
        c, d, xs = case(kind, taps, max_delay, blocks, taps + max_delay)
        same(product.sparse(kind, c, d, max_delay, xs), ref.sparse(kind, c, d, max_delay, xs))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_sparse_dropin_device_state(product, torch_gpu, ref, kind):
    """State buffer in device memory: the circular write and the tap reads happen on the GPU."""
    torch = torch_gpu
    tdt = {"f32": torch.float32, "q31": torch.int32, "q15": torch.int16, "q7": torch.int8}[kind]
    keep = []

    def dev_state(n, dt):
        t = torch.full((n,), 3, dtype=tdt, device="cuda")
        keep.append(t)
        return t.data_ptr(), lambda: t.cpu().numpy().copy()

    c, d, xs = case(kind, 16, 100, [64, 64, 64], 9)
    same(product.sparse(kind, c, d, 100, xs, state_mem=dev_state), ref.sparse(kind, c, d, 100, xs))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("taps,max_delay,block", [(32, 1000, 4096), (7, 20, 999), (12, 20000, 700), (2, 0, 5)])
def test_sparse_batch_bitexact(dsp, torch_gpu, ref, kind, taps, max_delay, block):
    """Batched device API: 5 streams, two consecutive calls each, d_hist carrying the last
    maxDelay samples (LDS-staged kernel; maxDelay = 20000 takes the direct-read kernel)."""
    torch = torch_gpu
    tdt = {"f32": torch.float32, "q31": torch.int32, "q15": torch.int16, "q7": torch.int8}[kind]
    batch = 5
    c, d, _ = case(kind, taps, max_delay, [1], taps * 3 + max_delay)
    streams = [case(kind, taps, max_delay, [block, block], 100 + i)[2] for i in range(batch)]
    dc = torch.from_numpy(c.copy()).cuda()
    dd = torch.from_numpy(d.copy()).cuda()
    S = _abi.arm_fir_sparse_instance(numTaps=taps, pCoeffs=dc.data_ptr(), maxDelay=max_delay, pTapDelay=dd.data_ptr())
    hist = torch.zeros((batch, max(max_delay, 1)), dtype=tdt, device="cuda")
    f = getattr(dsp.lib, f"arm_fir_sparse_{kind}_batch")
    got = []
    for k in range(2):
        src = torch.from_numpy(np.stack([streams[i][k] for i in range(batch)])).cuda()
        dst = torch.empty((batch, block), dtype=tdt, device="cuda")
        st = f(C.byref(S), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), block, batch,
               C.c_void_p(hist.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert st == 0, dsp.last_error()
        got.append(dst.cpu().numpy())
    h = hist.cpu().numpy()
    for i in range(batch):
        want, _, _ = ref.sparse(kind, c, d, max_delay, streams[i])
        for k in range(2):
            assert got[k][i].tobytes() == want[k].tobytes(), (i, k)
        tail = np.concatenate([np.zeros(max_delay, refs.DTYPE[kind]), streams[i][0], streams[i][1]])[-max_delay:]
        assert h[i, :max_delay].tobytes() == (tail.tobytes() if max_delay else b"")


@pytest.mark.gpu
def test_cmsisdsp_module_sparse(torch_gpu, ref):
    """The cmsisdsp-compatible module with the reference binding's call shapes
    (cmsisdsp_filtering.c: init "OhOOOh", blockSize = len(pState) - len(pCoeffs) + 1;
    arm_fir_sparse_f32(S, pSrc, pScratchIn))."""
    import cmsisdsp as d
    c, dl, xs = case("f32", 6, 40, [64, 64], 21)
    S = d.arm_fir_sparse_instance_f32()
    d.arm_fir_sparse_init_f32(S, 6, c, np.zeros(40 + 64 + 5), dl, 40)
    want = ref.sparse("f32", c, dl, 40, xs, block_size=64 + 5)[0]
    for x, w in zip(xs, want):
        assert d.arm_fir_sparse_f32(S, x, np.zeros(64)).tobytes() == w.tobytes()
    assert S.stateIndex() == 2 * 64 % (40 + 64)       # L = maxDelay + len(pSrc)
