"""GPU parity: batched and drop-in complex FFT (f32 / q31 / q15) vs the reference scalar C.

The bar is bit-exactness for every type (the f32 kernel replays the reference's
operation order with contraction off), checked against oracle/_ref (the reference's own
code) on seeded inputs, every supported length, both directions, bit reversal on/off.
Reference behaviour exercised: arm_cfft_f32.c:1243-1298, arm_cfft_q31.c:704-755,
arm_cfft_q15.c:671-722; test sizes follow Testing/desc.txt Transform suites (16..4096).
"""
import numpy as np
import pytest

import refs

pytestmark = pytest.mark.gpu

SIZES = [16, 32, 64, 128, 256, 512, 1024, 2048, 4096]
KINDS = ["f32", "q31", "q15"]
TORCH_DT = {"f32": "float32", "q31": "int32", "q15": "int16"}


def _dev(torch, arr, kind):
    return torch.from_numpy(arr.copy()).to("cuda")


def _batched(dsp, torch, kind, n, x, ifft, bitrev):
    S = dsp.const_instance(f"arm_cfft_sR_{kind}_len{n}")
    d = _dev(torch, x, kind)
    dsp.cfft_batch(S, d, ifft, bitrev)
    torch.cuda.synchronize()
    return d.cpu().numpy()


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("ifft,bitrev", [(0, 1), (1, 1), (0, 0), (1, 0)])
def test_cfft_batch_bitexact(dsp, torch_gpu, ref, kind, n, ifft, bitrev):
    batch = 37   # not a multiple of any workgroup's transform count: ragged last block
    dist = "uniform" if kind == "f32" else ("sine" if n % 3 else "uniform")
    x = np.stack([refs.rand_input(kind, 2 * n, seed=1000 * n + r + 7 * ifft + 3 * bitrev, dist=dist)
                  for r in range(batch)])
    want = ref.cfft_many(kind, n, x, ifft, bitrev)
    got = _batched(dsp, torch_gpu, kind, n, x, ifft, bitrev)
    if kind == "f32":
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
    else:
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("kind", ["q31", "q15"])
@pytest.mark.parametrize("n", [16, 32, 1024, 2048, 4096])
@pytest.mark.parametrize("dist", ["uniform", "extreme"])
def test_cfft_fixed_wrap_saturation(dsp, torch_gpu, ref, kind, n, dist):
    """Full-range and all-extreme words: int32 wrap, __SSAT and int16 truncation paths."""
    x = np.stack([refs.rand_input(kind, 2 * n, seed=77 + r, dist=dist) for r in range(5)])
    for ifft in (0, 1):
        np.testing.assert_array_equal(_batched(dsp, torch_gpu, kind, n, x, ifft, 1),
                                      ref.cfft_many(kind, n, x, ifft, 1))


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("n", [16, 256, 1024, 4096])
def test_cfft_dropin_host_pointer(dsp, torch_gpu, ref, kind, n):
    """The synchronous drop-in API on host memory (staged through the device; f32 N = 1024 one
    transform runs the 2-wave latency kernel, cfft_f32.hip cfft_f32_n1024_lat_kernel): every
    (ifftFlag, bitReverseFlag) pair, ifftFlag 2 = forward as in arm_cfft_f32.c:1252."""
    x = refs.rand_input(kind, 2 * n, seed=5 + n)
    for ifft, bitrev in [(0, 1), (1, 1), (0, 0), (1, 0), (2, 1)]:
        S = getattr(dsp, f"arm_cfft_instance_{kind}")()
        assert getattr(dsp, f"arm_cfft_init_{kind}")(S, n) == 0
        got = getattr(dsp, f"arm_cfft_{kind}")(S, x, ifft, bitrev)
        want = ref.cfft(kind, n, x, ifft, bitrev)
        assert got.tobytes() == want.tobytes()


def test_cfft_unsupported_length_is_noop(dsp, torch_gpu):
    """arm_cfft_f32.c:1263-1280: a length outside the switch leaves the buffer untouched."""
    S = dsp.arm_cfft_instance_f32()
    S.fftLen = 100
    x = np.arange(200, dtype=np.float32)
    assert np.array_equal(dsp.arm_cfft_f32(S, x, 0, 1), x)
    assert dsp.arm_cfft_init_f32(dsp.arm_cfft_instance_f32(), 100) == dsp.ARM_MATH_ARGUMENT_ERROR


def test_cfft_ifft_flag_semantics(dsp, torch_gpu, ref):
    """Only ifftFlag == 1 selects the inverse (arm_cfft_f32.c:1252); 2 is a forward transform."""
    x = refs.rand_input("f32", 2048, seed=3)
    got = _batched(dsp, torch_gpu, "f32", 1024, x[None], 2, 1)[0]
    assert got.tobytes() == ref.cfft("f32", 1024, x, 0, 1).tobytes()


def test_cfft_custom_bitrev_table(dsp, torch_gpu, ref):
    """A non-canonical swap table is honoured exactly (generic permutation path)."""
    import ctypes as C
    n = 64
    S = dsp.arm_cfft_instance_f32()
    dsp.arm_cfft_init_f32(S, n)
    tab = np.array([8 * 1, 8 * 5, 8 * 2, 8 * 9, 8 * 1, 8 * 2], dtype=np.uint16)   # overlapping swaps
    S.pBitRevTable = tab.ctypes.data_as(C.POINTER(C.c_uint16))
    S.bitRevLength = len(tab)
    x = refs.rand_input("f32", 2 * n, seed=9)
    got = dsp.arm_cfft_f32(S, x, 0, 1)
    Sr = ref.cfft_instance("f32", n)
    Sr.pBitRevTable = tab.ctypes.data_as(C.POINTER(C.c_uint16))
    Sr.bitRevLength = len(tab)
    buf = x.copy()
    ref.fn("arm_cfft_f32")(C.byref(Sr), buf.ctypes.data, 0, 1)
    assert got.tobytes() == buf.tobytes()


@pytest.mark.parametrize("kind,n", [("f32", 1024), ("q31", 4096), ("q15", 4096), ("f32", 4096)])
def test_cfft_batch_larger_than_resident_grid(dsp, torch_gpu, ref, kind, n):
    """Persistent kernels loop over the batch: a batch several times the resident grid."""
    batch = 9000 if n == 1024 else 2500
    x = np.stack([refs.rand_input(kind, 2 * n, seed=r) for r in range(batch)])
    for ifft in (0, 1):
        got = _batched(dsp, torch_gpu, kind, n, x, ifft, 1)
        want = ref.cfft_many(kind, n, x, ifft, 1)
        assert got.tobytes() == want.tobytes()
