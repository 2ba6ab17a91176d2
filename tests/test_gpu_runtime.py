"""GPU: the host runtime around the kernels — the multi-GPU C entry point, several host
threads sharing one device, in-place (aliased) FIR calls, aliased conv/correlate operands,
user tables whose contents change at a reused address, and the pinned host staging of the
drop-in API.  Every result is compared bit for bit with the reference scalar C
(oracle/_ref).  Reference call shapes: transform_functions.h:456-460 (arm_cfft_*),
filtering_functions.h:233-237 (arm_fir_f32), arm_correlate_f32.c:1013-1096."""
import ctypes as C
import threading

import numpy as np
import pytest

import refs

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ multi-GPU C entry point
@pytest.mark.parametrize("kind,n", [("f32", 1024), ("q31", 4096), ("q15", 4096), ("f32", 256)])
def test_cfft_batch_multi_bitexact(dsp, torch_gpu, ref, kind, n):
    """Shards over every visible device (two shards per device, ragged sizes): each shard
    equals the reference on its transforms."""
    torch = torch_gpu
    ndev = dsp.device_count()
    assert ndev == torch.cuda.device_count() and ndev >= 1
    counts = [5 + 3 * s for s in range(2 * ndev)]
    devs = [s % ndev for s in range(2 * ndev)]
    xs = [np.stack([refs.rand_input(kind, 2 * n, seed=100 * s + r) for r in range(c)]) for s, c in enumerate(counts)]
    shards = [torch.from_numpy(x.copy()).to(f"cuda:{d}") for x, d in zip(xs, devs)]
    S = dsp.const_instance(f"arm_cfft_sR_{kind}_len{n}")
    for ifft in (0, 1):
        for t, x in zip(shards, xs):
            t.copy_(torch.from_numpy(x))
        torch.cuda.synchronize()
        dsp.cfft_batch_multi(S, shards, ifft, 1)
        for t, x in zip(shards, xs):
            assert t.cpu().numpy().tobytes() == ref.cfft_many(kind, n, x, ifft, 1).tobytes()


def test_cfft_batch_multi_rejects_bad_shards(dsp, torch_gpu):
    torch = torch_gpu
    S = dsp.const_instance("arm_cfft_sR_f32_len1024")
    t = torch.zeros((2, 2048), device="cuda")
    ptrs = (C.c_void_p * 1)(t.data_ptr())
    cnts = (C.c_uint32 * 1)(2)
    bad = (C.c_int * 1)(dsp.device_count())                     # one past the last device
    assert dsp.lib.arm_cfft_f32_batch_multi(C.byref(S), 1, bad, ptrs, cnts, 0, 1) == dsp.ARM_MATH_ARGUMENT_ERROR
    null = (C.c_void_p * 1)(None)
    ok_dev = (C.c_int * 1)(0)
    assert dsp.lib.arm_cfft_f32_batch_multi(C.byref(S), 1, ok_dev, null, cnts, 0, 1) == dsp.ARM_MATH_ARGUMENT_ERROR
    assert dsp.lib.arm_cfft_f32_batch_multi(C.byref(S), 0, None, None, None, 0, 1) == dsp.ARM_MATH_SUCCESS
    assert torch.count_nonzero(t).item() == 0                   # nothing was launched


# ------------------------------------------------------------------ host threads
def test_four_host_threads_share_one_device(dsp, torch_gpu, ref):
    """Four host threads, each on its own HIP stream, call arm_cfft_f32_batch and
    arm_fir_f32_batch concurrently on device 0 (ctypes releases the GIL during the
    calls): the table cache, the per-thread scratch and the coefficient cache under
    contention.  Every thread's results stay bit-exact."""
    torch = torch_gpu
    n, batch, taps, block = 1024, 64, 32, 1000
    coeffs = [refs.rand_input("f32", taps, seed=900 + t) for t in range(4)]   # distinct host coefficient sets
    xs = [np.stack([refs.rand_input("f32", 2 * n, seed=40 * t + r) for r in range(batch)]) for t in range(4)]
    sig = [np.stack([refs.rand_input("f32", block, seed=70 * t + r) for r in range(8)]) for t in range(4)]
    want_fft = [ref.cfft_many("f32", n, x, 0, 1) for x in xs]
    want_fir = [np.stack([ref.fir("f32", coeffs[t], [sig[t][r]])[0][0] for r in range(8)]) for t in range(4)]
    errors, got_fft, got_fir = [], [None] * 4, [None] * 4
    S = dsp.const_instance("arm_cfft_sR_f32_len1024")

    def worker(t):
        try:
            torch.cuda.set_device(0)
            st = torch.cuda.Stream()
            fir = dsp.arm_fir_instance_f32()
            fir.numTaps = taps
            fir.pCoeffs = coeffs[t].ctypes.data_as(C.POINTER(C.c_float))   # host coefficients
            with torch.cuda.stream(st):
                d = torch.from_numpy(xs[t].copy()).cuda()
                src = torch.from_numpy(sig[t].copy()).cuda()
                dst = torch.empty_like(src)
                hist = torch.zeros((8, taps - 1), device="cuda")
                for _ in range(5):                                   # interleave many launches
                    d.copy_(torch.from_numpy(xs[t]))
                    dsp.cfft_batch(S, d, 0, 1, stream=st)
                    hist.zero_()
                    dsp.fir_batch(fir, src, dst, hist, stream=st)
                st.synchronize()
                got_fft[t] = d.cpu().numpy()
                got_fir[t] = dst.cpu().numpy()
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not errors, errors
    for t in range(4):
        assert got_fft[t].tobytes() == want_fft[t].tobytes()
        assert got_fir[t].tobytes() == want_fir[t].tobytes()


# ------------------------------------------------------------------ aliasing
def test_fir_dropin_in_place_on_device(dsp, torch_gpu, ref):
    """arm_fir_f32 with pSrc == pDst on the device, two calls: outputs, carried history and
    the state tail [history ; block input] equal the reference's (which copies each input
    into pState before writing pDst)."""
    torch = torch_gpu
    taps, block = 29, 700
    c = refs.rand_input("f32", taps, seed=1)
    blocks = [refs.rand_input("f32", block, seed=2 + k) for k in range(2)]
    want, want_state = ref.fir("f32", c, blocks)
    S = dsp.arm_fir_instance_f32()
    dc = torch.from_numpy(c).cuda()
    state = torch.full((taps + block - 1,), 7.0, device="cuda")
    dsp.lib.arm_fir_init_f32(C.byref(S), taps, C.c_void_p(dc.data_ptr()), C.c_void_p(state.data_ptr()), block)
    for k in range(2):
        buf = torch.from_numpy(blocks[k].copy()).cuda()
        dsp.lib.arm_fir_f32(C.byref(S), C.c_void_p(buf.data_ptr()), C.c_void_p(buf.data_ptr()), block)
        dsp._check_void("arm_fir_f32")
        assert buf.cpu().numpy().tobytes() == want[k].tobytes()
    assert state.cpu().numpy().tobytes() == want_state.tobytes()


@pytest.mark.parametrize("kind", ["f32", "q15", "q31"])
def test_fir_batch_in_place(dsp, torch_gpu, ref, kind):
    """arm_fir_*_batch with d_src == d_dst over two calls (several chunks per filter)."""
    torch = torch_gpu
    taps = 40 if kind == "q15" else 37
    block, batch = 5000, 6
    c = refs.rand_input(kind, taps, seed=11)
    blocks = [[refs.rand_input(kind, block, seed=50 * f + k) for k in range(2)] for f in range(batch)]
    want = [ref.fir(kind, c, blocks[f])[0] for f in range(batch)]
    S = getattr(dsp, f"arm_fir_instance_{kind}")()
    S.numTaps = taps
    dc = torch.from_numpy(c.copy()).cuda()
    S.pCoeffs = C.cast(dc.data_ptr(), S._fields_[2][1])
    hist = torch.zeros((batch, taps - 1), dtype=dc.dtype, device="cuda")
    for k in range(2):
        buf = torch.from_numpy(np.stack([blocks[f][k] for f in range(batch)])).cuda()
        dsp.fir_batch(S, buf, buf, hist, kind=kind)
        torch.cuda.synchronize()
        got = buf.cpu().numpy()
        for f in range(batch):
            assert got[f].tobytes() == want[f][k].tobytes(), (k, f)


@pytest.mark.parametrize("fn", ["correlate_f32", "correlate_q15", "correlate_q31", "conv_fast_q15",
                                "conv_fast_q31", "correlate_fast_q31"])
def test_conv_family_same_base_pointer_shorter_first(dsp, torch_gpu, ref, fn):
    """pSrcA and pSrcB share one base address with srcALen < srcBLen (e.g.
    arm_correlate_f32(x, 5, x, 10)): the operand swap must follow the lengths, not the
    pointers.  Drop-in (host and device pointers) and batched."""
    torch = torch_gpu
    x = refs.rand_input(fn[-3:], 300, seed=3)
    for la, lb in ((5, 10), (17, 250)):
        want, _ = ref.conv_family(fn, x[:la], x[:lb], fill=0)
        got, _ = dsp.arm_conv_family(fn, x[:la], x[:lb], fill=0)
        assert got.tobytes() == want.tobytes(), (la, lb)
        d = torch.from_numpy(x.copy()).cuda()
        n = len(want)
        out = torch.zeros(n, dtype=d.dtype, device="cuda")
        getattr(dsp.lib, f"arm_{fn}")(C.c_void_p(d.data_ptr()), la, C.c_void_p(d.data_ptr()), lb,
                                      C.c_void_p(out.data_ptr()))
        dsp._check_void(fn)
        assert out.cpu().numpy().tobytes() == want.tobytes(), (la, lb)
        outb = torch.zeros((1, n), dtype=d.dtype, device="cuda")
        dsp.conv_family_batch(fn, d[:la].view(1, la), d[:lb].view(1, lb), outb)
        torch.cuda.synchronize()
        assert outb[0].cpu().numpy().tobytes() == want.tobytes(), (la, lb)


# ------------------------------------------------------------------ user tables by content
def test_user_tables_follow_their_contents(dsp, torch_gpu, ref):
    """A user twiddle table and a user bit-reversal table are rewritten IN PLACE between two
    calls (same address, new words): the second call must use the new words."""
    n = 64
    tw = np.ctypeslib.as_array(C.cast(dsp.const_instance("arm_cfft_sR_f32_len64").pTwiddle,
                                      C.POINTER(C.c_float)), (2 * n,)).copy()
    tab = np.array([8 * 1, 8 * 5, 8 * 2, 8 * 9], dtype=np.uint16)
    x = refs.rand_input("f32", 2 * n, seed=21)
    for variant in range(2):
        if variant:                       # new contents at the same addresses
            tw[1::2] *= -1.0              # conjugate twiddles: a different (but valid) transform
            tab[:] = [8 * 3, 8 * 7, 8 * 4, 8 * 60]
        S = dsp.arm_cfft_instance_f32()
        dsp.arm_cfft_init_f32(S, n)
        S.pTwiddle = tw.ctypes.data_as(C.POINTER(C.c_float))
        S.pBitRevTable = tab.ctypes.data_as(C.POINTER(C.c_uint16))
        S.bitRevLength = len(tab)
        got = dsp.arm_cfft_f32(S, x, 0, 1)
        Sr = ref.cfft_instance("f32", n)
        Sr.pTwiddle = tw.ctypes.data_as(C.POINTER(C.c_float))
        Sr.pBitRevTable = tab.ctypes.data_as(C.POINTER(C.c_uint16))
        Sr.bitRevLength = len(tab)
        buf = x.copy()
        ref.fn("arm_cfft_f32")(C.byref(Sr), buf.ctypes.data, 0, 1)
        assert got.tobytes() == buf.tobytes(), variant


def test_device_resident_twiddles_used_in_place(dsp, torch_gpu, ref):
    """An instance whose twiddle table is a device pointer is used without a copy, and a
    change of those device words is seen by the next call."""
    torch = torch_gpu
    import ctypes
    n = 1024
    base = dsp.const_instance("arm_cfft_sR_f32_len1024")
    host_tw = np.ctypeslib.as_array(ctypes.cast(base.pTwiddle, ctypes.POINTER(ctypes.c_float)), (2 * n,)).copy()
    dtw = torch.from_numpy(host_tw.copy()).cuda()
    S = dsp.arm_cfft_instance_f32()
    dsp.arm_cfft_init_f32(S, n)
    S.pTwiddle = ctypes.cast(dtw.data_ptr(), ctypes.POINTER(ctypes.c_float))
    x = np.stack([refs.rand_input("f32", 2 * n, seed=s) for s in range(3)])
    for variant in range(2):
        if variant:
            dtw[1::2] *= -1.0
            host_tw[1::2] *= -1.0
        d = torch.from_numpy(x.copy()).cuda()
        dsp.cfft_batch(S, d, 0, 1)
        torch.cuda.synchronize()
        Sr = ref.cfft_instance("f32", n)
        Sr.pTwiddle = host_tw.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
        want = np.stack([_ref_cfft(ref, Sr, r) for r in x])
        assert d.cpu().numpy().tobytes() == want.tobytes(), variant


def _ref_cfft(ref, S, row):
    buf = row.copy()
    ref.fn("arm_cfft_f32")(C.byref(S), buf.ctypes.data, 0, 1)
    return buf


# ------------------------------------------------------------------ pinned staging
def test_dropin_pinned_staging_repeated_sizes(dsp, torch_gpu, ref):
    """The drop-in host path reuses its pinned bounce buffers across calls of growing and
    shrinking sizes without mixing up words."""
    for n in (4096, 16, 1024, 64, 4096):
        x = refs.rand_input("q31", 2 * n, seed=n)
        S = dsp.arm_cfft_instance_q31()
        dsp.arm_cfft_init_q31(S, n)
        assert dsp.arm_cfft_q31(S, x, 0, 1).tobytes() == ref.cfft("q31", n, x, 0, 1).tobytes()
    a = refs.rand_input("f32", 40 * 33, seed=1).reshape(40, 33)
    b = refs.rand_input("f32", 33 * 21, seed=2).reshape(33, 21)
    st, c = dsp.arm_mat_mult_f32(a, b)
    assert st == 0
    np.testing.assert_allclose(c, a.astype(np.float64) @ b.astype(np.float64), rtol=1e-5, atol=1e-5)


# ------------------------------------------------------------------ table cache bound
def test_coefficient_cache_stays_bounded(dsp, torch_gpu, ref):
    """Fresh coefficients on every call (a time-varying filter) go through the content-keyed
    cache; with a 1 MiB limit the cache cycles instead of growing, results stay bit-exact, and
    the device memory the process holds stays flat."""
    torch = torch_gpu
    rng = np.random.default_rng(3)
    taps, block = 1024, 64                       # 4 KiB of taps per call
    dsp.set_table_cache_limit(1 << 20)
    try:
        x = rng.uniform(-1, 1, block).astype(np.float32)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info()[0]
        for i in range(600):                     # 2.4 MiB of distinct coefficient sets
            c = rng.standard_normal(taps).astype(np.float32)
            f = dsp.FirF32(c, block)
            got = f(x)
            if i % 97 == 0:
                want, _ = ref.fir("f32", c, [x])
                assert got.tobytes() == want[0].tobytes()
            assert dsp.table_cache_bytes() <= 1 << 20
        torch.cuda.synchronize()
        assert free0 - torch.cuda.mem_get_info()[0] < 64 << 20
    finally:
        dsp.set_table_cache_limit(256 << 20)


def test_cfft_batch_multi_orders_after_torch_work(dsp, torch_gpu, ref):
    """Shards written by torch kernels still in flight (no explicit synchronize): the wrapper
    orders the library's streams after them."""
    torch = torch_gpu
    n, rows = 1024, 64
    x = np.stack([refs.rand_input("f32", 2 * n, seed=500 + r) for r in range(rows)])
    src = torch.from_numpy(x).cuda()
    S = dsp.const_instance("arm_cfft_sR_f32_len1024")
    for _ in range(3):
        shard = torch.zeros_like(src)
        for _ in range(20):                      # queue enough torch work to still be running
            shard.mul_(0.5)
        shard.copy_(src)
        dsp.cfft_batch_multi(S, [shard], 0, 1)
        assert shard.cpu().numpy().tobytes() == ref.cfft_many("f32", n, x, 0, 1).tobytes()


# ------------------------------------------------------------------ zero-copy drop-in staging
def test_dropin_zero_copy_fresh_every_call(dsp, torch_gpu, ref):
    """Small host-pointer calls run the kernel on a coherent pinned copy (no DMA): 40
    consecutive arm_cfft_q31 / arm_cfft_f32 calls on fresh data reuse the same staging slot and
    must never see a previous call's words."""
    rng = np.random.default_rng(9)
    for kind, n in (("f32", 1024), ("q31", 4096), ("q15", 256)):
        S = dsp.const_instance(f"arm_cfft_sR_{kind}_len{n}")
        fn = {"f32": dsp.arm_cfft_f32, "q31": dsp.arm_cfft_q31, "q15": dsp.arm_cfft_q15}[kind]
        for i in range(40):
            x = refs.rand_input(kind, 2 * n, seed=int(rng.integers(1 << 30)))
            got = fn(S, x.copy(), i & 1, 1)
            assert np.asarray(got).tobytes() == ref.cfft(kind, n, x, i & 1, 1).tobytes(), (kind, i)


@pytest.mark.parametrize("taps,block", [(29, 32), (64, 10), (300, 7), (2, 1)])
def test_dropin_fir_zero_copy_short_blocks(dsp, torch_gpu, ref, taps, block):
    """Blocks shorter than the history (the new history reaches into the old one) and many
    calls in a row through the zero-copy path: outputs and the caller's state buffer."""
    rng = np.random.default_rng(taps * 31 + block)
    c = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
    blocks = [rng.uniform(-1, 1, block).astype(np.float32) for _ in range(25)]
    f = dsp.FirF32(c, block)
    want, state = ref.fir("f32", c, blocks)
    for b, w in zip(blocks, want):
        assert f(b).tobytes() == w.tobytes()
    assert f.state.tobytes() == state.tobytes()


# ------------------------------------------------------------------ multi-GPU FIR / mat_mult
@pytest.mark.parametrize("kind", ["f32", "q15", "fast_q15", "q31", "fast_q31", "q7"])
def test_fir_batch_multi_bitexact(dsp, torch_gpu, ref, kind):
    """arm_fir_*_batch_multi: filters sharded with their history rows over every visible device
    (two ragged shards per device), two calls with state carry, host coefficients (uploaded per
    device): every filter equals the reference's stream."""
    torch = torch_gpu
    base = kind.split("_")[-1]
    ndev = dsp.device_count()
    taps, block = (64 if base == "q15" else 37), 777
    c = refs.rand_input(base, taps, seed=5)
    counts = [3 + 2 * s for s in range(2 * ndev)]
    devs = [s % ndev for s in range(2 * ndev)]
    blocks = [[[refs.rand_input(base, block, seed=1000 * s + 10 * f + k) for k in range(2)] for f in range(cnt)]
              for s, cnt in enumerate(counts)]
    S = {"f32": dsp.arm_fir_instance_f32, "q15": dsp.arm_fir_instance_q15, "q31": dsp.arm_fir_instance_q31,
         "q7": dsp.arm_fir_instance_q7}[base]()
    S.numTaps = taps
    S.pCoeffs = C.cast(c.ctypes.data, S._fields_[2][1])
    dt = {"f32": torch.float32, "q15": torch.int16, "q31": torch.int32, "q7": torch.int8}[base]
    hists = [torch.zeros((cnt, taps - 1), dtype=dt, device=f"cuda:{d}") for cnt, d in zip(counts, devs)]
    for k in range(2):
        shards = []
        for s, (cnt, d) in enumerate(zip(counts, devs)):
            src = torch.from_numpy(np.stack([blocks[s][f][k] for f in range(cnt)])).to(f"cuda:{d}")
            shards.append((src, torch.empty_like(src), hists[s]))
        dsp.fir_batch_multi(S, shards, kind=kind)
        for s, (src, dst, _) in enumerate(shards):
            got = dst.cpu().numpy()
            for f in range(counts[s]):
                want, _ = ref.fir(kind, c, blocks[s][f][:k + 1])
                assert got[f].tobytes() == want[k].tobytes(), (s, f, k)


@pytest.mark.parametrize("dtype", ["f32", "q15", "q31"])
def test_mat_mult_batch_multi_bitexact(dsp, torch_gpu, ref, oracle, dtype):
    """arm_mat_mult_*_batch_multi over every visible device: f32 equals the fmaf-chain
    restatement bit for bit, q15 / q31 the reference."""
    torch = torch_gpu
    ndev = dsp.device_count()
    m, k, n = 65, 70, 33
    counts = [2 + s for s in range(2 * ndev)]
    devs = [s % ndev for s in range(2 * ndev)]
    rng = np.random.default_rng(7)
    shards, host = [], []
    for cnt, d in zip(counts, devs):
        if dtype == "f32":
            a = rng.uniform(-1, 1, (cnt, m, k)).astype(np.float32)
            b = rng.uniform(-1, 1, (cnt, k, n)).astype(np.float32)
        else:
            bits, npdt = (15, np.int16) if dtype == "q15" else (31, np.int32)
            a = rng.integers(-(1 << bits), 1 << bits, (cnt, m, k)).astype(npdt)
            b = rng.integers(-(1 << bits), 1 << bits, (cnt, k, n)).astype(npdt)
        ta, tb = torch.from_numpy(a).to(f"cuda:{d}"), torch.from_numpy(b).to(f"cuda:{d}")
        tc = torch.empty((cnt, m, n), dtype=ta.dtype, device=f"cuda:{d}")
        shards.append((ta, tb, tc))
        host.append((a, b))
    dsp.mat_mult_batch_multi(shards)
    for (a, b), (_, _, tc) in zip(host, shards):
        got = tc.cpu().numpy()
        for i in range(a.shape[0]):
            want = oracle.mat_mult_fmaf(a[i], b[i])[1] if dtype == "f32" else ref.mat_mult_fixed(dtype, a[i], b[i])[1]
            assert got[i].tobytes() == want.tobytes(), i


# ------------------------------------------------------------------ cache eviction under load
def test_table_cache_eviction_two_threads(dsp, torch_gpu, ref):
    """two host threads with a 64 KiB table-cache limit.  Each calls the
    drop-in arm_cfft_f32 with a custom bit-reversal table AND user twiddles that change every
    call (two content-cached blobs per call, which must not evict each other), and queues
    arm_fir_f32_batch with fresh host coefficients per call on its own stream without waiting
    (evicted coefficient sets may still be read by queued kernels: they must be released only
    after them).  Every result is bit-exact."""
    torch = torch_gpu
    n, taps, block, batch, iters = 64, 256, 512, 2, 120
    base_tw = np.ctypeslib.as_array(C.cast(dsp.const_instance("arm_cfft_sR_f32_len64").pTwiddle,
                                           C.POINTER(C.c_float)), (2 * n,)).copy()
    tab = np.array([8 * 3, 8 * 7, 8 * 4, 8 * 60, 8 * 1, 8 * 5], dtype=np.uint16)
    errors = []
    results = [dict() for _ in range(2)]
    dsp.set_table_cache_limit(64 << 10)
    try:
        def worker(t):
            try:
                torch.cuda.set_device(0)
                rng = np.random.default_rng(100 + t)
                st = torch.cuda.Stream()
                xs = rng.uniform(-1, 1, (batch, block)).astype(np.float32)
                fir_in = torch.from_numpy(xs).cuda()
                outs, cs, fft = [], [], []
                keep = []
                with torch.cuda.stream(st):
                    for i in range(iters):
                        tw = (base_tw * rng.uniform(0.5, 1.5, 2 * n)).astype(np.float32)   # new contents
                        x = rng.uniform(-1, 1, 2 * n).astype(np.float32)
                        S = dsp.arm_cfft_instance_f32()
                        dsp.arm_cfft_init_f32(S, n)
                        S.pTwiddle = tw.ctypes.data_as(C.POINTER(C.c_float))
                        S.pBitRevTable = tab.ctypes.data_as(C.POINTER(C.c_uint16))
                        S.bitRevLength = len(tab)
                        fft.append((tw, x, dsp.arm_cfft_f32(S, x, i & 1, 1)))
                        c = rng.standard_normal(taps).astype(np.float32)
                        fir = dsp.arm_fir_instance_f32()
                        fir.numTaps = taps
                        fir.pCoeffs = c.ctypes.data_as(C.POINTER(C.c_float))
                        dst = torch.empty_like(fir_in)
                        hist = torch.zeros((batch, taps - 1), device="cuda")
                        dsp.fir_batch(fir, fir_in, dst, hist, stream=st)   # no wait
                        outs.append(dst)
                        cs.append(c)
                        keep.append(hist)
                    st.synchronize()
                results[t] = {"fft": fft, "fir": [(c, o.cpu().numpy()) for c, o in zip(cs, outs)], "x": xs}
            except Exception as e:   # noqa: BLE001 - reported below
                errors.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=300)
        assert not errors, errors
        assert dsp.table_cache_bytes() <= 64 << 10
    finally:
        dsp.set_table_cache_limit(256 << 20)
    for t in range(2):
        for i, (tw, x, got) in enumerate(results[t]["fft"]):
            Sr = ref.cfft_instance("f32", n)
            Sr.pTwiddle = tw.ctypes.data_as(C.POINTER(C.c_float))
            Sr.pBitRevTable = tab.ctypes.data_as(C.POINTER(C.c_uint16))
            Sr.bitRevLength = len(tab)
            buf = x.copy()
            ref.fn("arm_cfft_f32")(C.byref(Sr), buf.ctypes.data, i & 1, 1)
            assert np.asarray(got).tobytes() == buf.tobytes(), (t, i)
        xs = results[t]["x"]
        for i, (c, got) in enumerate(results[t]["fir"]):
            if i % 7 and i != len(results[t]["fir"]) - 1:
                continue                              # every 7th set and the last against the reference
            for f in range(batch):
                want, _ = ref.fir("f32", c, [xs[f]])
                assert got[f].tobytes() == want[0].tobytes(), (t, i, f)


# ------------------------------------------------------------------ per-thread resources
def test_short_lived_threads_release_their_resources(dsp, torch_gpu, ref):
    """256 short-lived host threads, each making one host-pointer
    arm_cfft_f32 N=1024 call, one arm_fir_f32 29 x 32 call and one device arm_cfft_q31_batch
    call.  Every result equals the reference build's; afterwards no thread holds runtime
    resources (streams, scratch, staging, completion words are released at thread exit) and the
    device's free memory is back within 2 MiB.  The reference allocates nothing
    (arm_fir_f32.c:911-1280, arm_cfft_f32.c:1243-1298: SURVEY §8b "Ownership")."""
    torch = torch_gpu
    nthreads, wave = 256, 16
    S = dsp.const_instance("arm_cfft_sR_f32_len1024")
    Sq = dsp.const_instance("arm_cfft_sR_q31_len4096")
    taps, block = 29, 32
    coeffs = refs.rand_input("f32", taps, seed=5)
    xs = [refs.rand_input("f32", 2048, seed=1000 + t) for t in range(nthreads)]
    sig = [refs.rand_input("f32", block, seed=3000 + t) for t in range(nthreads)]
    qs = [refs.rand_input("q31", 8192, seed=5000 + t)[None, :] for t in range(nthreads)]
    want_fft = [ref.cfft_many("f32", 1024, x[None, :], 0, 1)[0] for x in xs]
    want_fir = [ref.fir("f32", coeffs, [s])[0][0] for s in sig]
    want_q = [ref.cfft_many("q31", 4096, q, 0, 1) for q in qs]
    dq = [torch.from_numpy(q.copy()).cuda() for q in qs]            # device buffers made up front
    # warm the main thread and the process-wide caches (tables, coefficient blob, events)
    dsp.arm_cfft_f32(S, xs[0], 0, 1)
    dsp.FirF32(coeffs, block)(sig[0])
    torch.cuda.synchronize()
    owners0 = dsp.thread_resource_owners()
    got_fft, got_fir, errors = [None] * nthreads, [None] * nthreads, []

    def worker(t):
        try:
            got_fft[t] = dsp.arm_cfft_f32(S, xs[t], 0, 1)
            got_fir[t] = dsp.FirF32(coeffs, block)(sig[t])
            dsp.cfft_batch(Sq, dq[t], 0, 1)
            torch.cuda.current_stream().synchronize()
        except Exception as e:   # noqa: BLE001 - reported below
            errors.append(repr(e))

    import time

    def settle():
        # Thread.join() returns when the Python body has finished; the OS thread runs its
        # thread_local destructors (where the release happens) just after
        t_end = time.monotonic() + 10.0
        while dsp.thread_resource_owners() != owners0 and time.monotonic() < t_end:
            time.sleep(0.01)
        torch.cuda.synchronize()
        return torch.cuda.mem_get_info()[0]

    free = []
    for w0 in range(0, nthreads, wave):
        th = [threading.Thread(target=worker, args=(t,)) for t in range(w0, w0 + wave)]
        for x in th:
            x.start()
        for x in th:
            x.join(timeout=120)
        assert not any(x.is_alive() for x in th)
        free.append(settle())
        assert dsp.thread_resource_owners() == owners0, (w0, dsp.thread_resource_owners(), owners0)
    assert not errors, errors
    # The first wave of 16 concurrent threads may make the HIP runtime create its pooled hardware
    # queues (process-wide, kept by the runtime); after it, 240 more threads must not move the
    # device's free memory: a per-thread leak would grow with every wave.
    assert abs(free[-1] - free[0]) <= (2 << 20), free
    for t in range(nthreads):
        assert got_fft[t].tobytes() == want_fft[t].tobytes(), t
        assert got_fir[t].tobytes() == want_fir[t].tobytes(), t
        assert dq[t].cpu().numpy().tobytes() == want_q[t].tobytes(), t


def test_release_thread_resources_then_call_again(dsp, torch_gpu, ref):
    """arm_mi355x_release_thread_resources() on the calling (main) thread drops its set; the next
    drop-in call re-creates what it needs and stays bit-exact."""
    S = dsp.const_instance("arm_cfft_sR_f32_len1024")
    x = refs.rand_input("f32", 2048, seed=77)
    want = ref.cfft_many("f32", 1024, x[None, :], 1, 1)[0]
    assert dsp.arm_cfft_f32(S, x, 1, 1).tobytes() == want.tobytes()
    n0 = dsp.thread_resource_owners()
    assert n0 >= 1
    dsp.release_thread_resources()
    assert dsp.thread_resource_owners() == n0 - 1
    assert dsp.arm_cfft_f32(S, x, 1, 1).tobytes() == want.tobytes()
    assert dsp.thread_resource_owners() == n0
