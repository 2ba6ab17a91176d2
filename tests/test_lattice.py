"""FIR lattice: arm_fir_lattice_{f32,q31,q15} (+ inits and the batched device API).

CPU: the oracle restatement (oracle/src/oracle_multirate.c) equals the reference build
(oracle/_ref, Source/FilteringFunctions/arm_fir_lattice_*.c, arm_fir_lattice_init_*.c) bit for
bit: outputs of consecutive calls and the final state, over stage counts and block sizes that
hit the reference's 4-sample / 4-stage unrolled loops and their remainders, full-range and
all-minimum fixed-point words (q31 wrap, q15 saturation).
GPU: the product (drop-in through host and device buffers; the batched device API over
several streams and two calls each, states carried on the device) equals the reference
build, including blocks spanning many segments (the segment-overlap path) and a stage count
above the segment limit (the sequential path).
"""
import ctypes as C

import numpy as np
import pytest

import refs
from cmsisdsp_amd import _abi

KINDS = ["f32", "q31", "q15"]
# (numStages, block sizes)
CASES = [(1, [16, 5]), (2, [7, 9]), (5, [64, 64, 3]), (8, [4096, 4096]), (33, [1000, 1023, 1]), (100, [3000, 50]),
         (255, [2100])]


def data(kind, n, rng, dist="full"):
    if kind == "f32":
        return rng.standard_normal(n).astype(np.float32)
    info = np.iinfo(refs.DTYPE[kind])
    if dist == "min":
        return np.full(n, info.min, refs.DTYPE[kind])
    return rng.integers(info.min, info.max, n, endpoint=True).astype(refs.DTYPE[kind])


def case(kind, stages, blocks, seed, dist="full"):
    rng = np.random.default_rng(seed)
    c = data(kind, stages, rng, dist)
    if kind == "f32":
        c = (rng.uniform(-0.9, 0.9, stages)).astype(np.float32)
    return c, [data(kind, b, rng, dist) for b in blocks]


def same(a, b):
    ya, sa = a
    yb, sb = b
    assert len(ya) == len(yb)
    for k, (u, v) in enumerate(zip(ya, yb)):
        assert u.tobytes() == v.tobytes(), k
    assert sa.tobytes() == sb.tobytes()


# ------------------------------------------------------------------ CPU: oracle == reference
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("stages,blocks", CASES)
def test_lattice_oracle_equals_reference(oracle, ref, kind, stages, blocks):
    c, xs = case(kind, stages, blocks, stages * 13 + len(blocks))
    same(oracle.lattice(kind, c, xs), ref.lattice(kind, c, xs))


@pytest.mark.parametrize("kind", ["q31", "q15"])
def test_lattice_extreme_words(oracle, ref, kind):
    """All-minimum samples and coefficients: q31 wraps, q15 saturates at every stage."""
    c, xs = case(kind, 12, [64, 64], 3, dist="min")
    same(oracle.lattice(kind, c, xs), ref.lattice(kind, c, xs))


# ------------------------------------------------------------------ GPU parity
@pytest.fixture(scope="module")
def product(dsp):
    return refs.Host(dsp.lib, "")


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_lattice_dropin_bitexact(product, torch_gpu, ref, kind):
    for stages, blocks in CASES + [(600, [700, 300])]:
        c, xs = case(kind, stages, blocks, stages + 1)
        same(product.lattice(kind, c, xs), ref.lattice(kind, c, xs))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
def test_lattice_dropin_device_state(product, torch_gpu, ref, kind):
    torch = torch_gpu
    tdt = {"f32": torch.float32, "q31": torch.int32, "q15": torch.int16}[kind]
    keep = []

    def dev_state(n, dt):
        t = torch.full((n,), 3, dtype=tdt, device="cuda")
        keep.append(t)
        return t.data_ptr(), lambda: t.cpu().numpy().copy()

    c, xs = case(kind, 20, [3000, 3000], 9)
    same(product.lattice(kind, c, xs, state_mem=dev_state), ref.lattice(kind, c, xs))


@pytest.mark.gpu
@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("stages,block", [(32, 4096), (7, 999), (511, 5000), (600, 300), (1, 1)])
def test_lattice_batch_bitexact(dsp, torch_gpu, ref, kind, stages, block):
    """Batched device API: 5 streams, two consecutive calls each, states on the device."""
    torch = torch_gpu
    tdt = {"f32": torch.float32, "q31": torch.int32, "q15": torch.int16}[kind]
    batch = 5
    c, _ = case(kind, stages, [1], stages * 3 + block)
    streams = [case(kind, stages, [block, block], 100 + i)[1] for i in range(batch)]
    dc = torch.from_numpy(c.copy()).cuda()
    S = _abi.arm_fir_lattice_instance(numStages=stages, pState=None, pCoeffs=dc.data_ptr())
    state = torch.zeros((batch, stages), dtype=tdt, device="cuda")
    f = getattr(dsp.lib, f"arm_fir_lattice_{kind}_batch")
    got = []
    for k in range(2):
        src = torch.from_numpy(np.stack([streams[i][k] for i in range(batch)])).cuda()
        dst = torch.empty((batch, block), dtype=tdt, device="cuda")
        st = f(C.byref(S), C.c_void_p(src.data_ptr()), C.c_void_p(dst.data_ptr()), block, batch,
               C.c_void_p(state.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert st == 0, dsp.last_error()
        got.append(dst.cpu().numpy())
    h = state.cpu().numpy()
    for i in range(batch):
        want, wstate = ref.lattice(kind, c, streams[i])
        for k in range(2):
            assert got[k][i].tobytes() == want[k].tobytes(), (i, k)
        assert h[i].tobytes() == wstate.tobytes()


@pytest.mark.gpu
def test_cmsisdsp_module_lattice(torch_gpu, ref):
    """cmsisdsp_filtering.c: arm_fir_lattice_init_f32 ("OhOO": S, numStages, pCoeffs, pState),
    arm_fir_lattice_f32(S, pSrc) -> pDst."""
    import cmsisdsp as d
    c, xs = case("f32", 6, [100, 37], 21)
    S = d.arm_fir_lattice_instance_f32()
    d.arm_fir_lattice_init_f32(S, 6, c, np.zeros(6))
    want = ref.lattice("f32", c, xs)[0]
    for x, w in zip(xs, want):
        assert d.arm_fir_lattice_f32(S, x).tobytes() == w.tobytes()
