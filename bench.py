#!/usr/bin/env python3
"""Benchmark of the MI355X CMSIS-DSP backend — the BASELINE.json headline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload WL] [--batch B]

Default workload (BASELINE.json configs[1]): batched arm_cfft_f32, fftLen 1024,
2^20 transforms per GPU (8 GiB in HBM, in place), bitReverseFlag 1; a step is one pass
of the hot path over the batch, alternating forward / inverse (the inverse rescales by
1/N, so values stay bounded).  The metric is whole-job complex samples per second.
The same line carries the q31 N=4096 bit-exact companion measurement, the roofline of
the dominant kernel (HIP-event average launch duration on the launch stream) and the
reference scalar C timed on this host's cores (cpu_baseline).

N > 1: launched by torch.distributed.run, one process per GPU; every rank processes its
own 2^20 transforms (weak scaling, no data-path collective), timed between barriers,
MAX over ranks.  Other workloads: cfft_q31_4096, cfft_q15_4096, fir_f32, fir_q15, mat_mult_f32,
mfcc_f32 (arm_mfcc_f32, fftLen 1024, the reference suite's 20-Mel/13-DCT tables).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cmsis-dsp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cmsisdsp_amd as dsp  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3     # dense f32 MFMA / packed-FMA VALU peak
FP32_NOFMA_TFLOPS = 78.6     # separate v_mul_f32 + v_add_f32 (bit-exact FIR)
METRIC = "Gsamples/sec batched arm_cfft_f32 N=1024 (+ q31 bit-exact) at 1/2/4/8 GPU"

WORKLOADS = {
    # name: (kind, fftLen / taps, default batch per GPU, algorithmic bytes per sample)
    "cfft_f32_1024": ("f32", 1024, 1 << 20, 16),
    "cfft_q31_4096": ("q31", 4096, 1 << 18, 16),
    "cfft_q15_4096": ("q15", 4096, 1 << 18, 8),
    "fir_f32": ("fir_f32", 128, 1 << 16, 8),
    "fir_q15": ("fir_q15", 128, 1 << 16, 4),
    "fir_q31": ("fir_q31", 128, 1 << 16, 8),
    "fir_fast_q15": ("fir_fast_q15", 128, 1 << 16, 4),
    "fir_fast_q31": ("fir_fast_q31", 128, 1 << 16, 8),
    "mat_mult_f32": ("mat", 1024, 256, None),
    "mfcc_f32": ("mfcc", 1024, 1 << 18, 4),
    "rfft_f32": ("rfft", 1024, 1 << 20, 8),
    # real length 8192 (inner CFFT 4096 = the fixed-point specialist); bytes per sample:
    # N words in, N words written back (the inner CFFT overwrites pSrc), 2N words out
    "rfft_q31": ("rfftq31", 8192, 1 << 16, 16),
    "rfft_q15": ("rfftq15", 8192, 1 << 16, 8),
    "conv_f32": ("conv", 128, 1 << 16, 8),
    "mat_mult_q15": ("matq15", 1024, 64, None),
    "mat_mult_q31": ("matq31", 1024, 64, None),
    "mat_mult_fast_q31": ("matfast_q31", 1024, 64, None),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ------------------------------------------------------------------ distributed plumbing
from cmsisdsp_amd import parallel  # noqa: E402

WORLD = parallel.World()


def barrier(world):
    parallel.barrier(WORLD)


def allreduce_max(x, world):
    return parallel.reduce_max(WORLD, x)


# ------------------------------------------------------------------ data + checkers
def synth(kind, n_words, rank, salt=0):
    """Deterministic synthetic input, rank-local (no scatter): uniform[-0.5,0.5) f32 or
    full-range integers from a per-rank generator (parallel.seed_for)."""
    g = torch.Generator(device="cuda")
    g.manual_seed(parallel.seed_for(rank, salt))
    if kind == "f32":
        return torch.rand(n_words, generator=g, device="cuda", dtype=torch.float32) - 0.5
    hi = 1 << (31 if kind == "q31" else 15)
    dt = torch.int32 if kind == "q31" else torch.int16
    return torch.randint(-hi, hi, (n_words,), generator=g, device="cuda", dtype=torch.int64).to(dt)


def cpu_checker():
    """The reference scalar C (oracle/_ref) if present, else the restatement (oracle/_build)."""
    import refs
    try:
        return refs.ref_lib(), "reference"
    except (FileNotFoundError, OSError):
        return refs.oracle_lib(), "port"


def flag_sequence(steps):
    return [s & 1 for s in range(steps)]            # fwd, inv, fwd, ...


# ------------------------------------------------------------------ CPU baseline
def cpu_baseline(workload, n):
    """Reference C on this host's cores, bounded sample (~16 thread-seconds)."""
    threads = min(16, os.cpu_count() or 1)
    secs = 1.0
    exe_ref = os.path.join(ROOT, "oracle", "_ref", "bench_ref")
    exe_port = os.path.join(ROOT, "oracle", "_build", "bench_port")
    exe, kind = (exe_ref, "reference") if os.path.exists(exe_ref) else (exe_port, "port")
    if not os.path.exists(exe):
        return None
    wl = {"cfft_f32_1024": "cfft_f32", "cfft_q31_4096": "cfft_q31", "cfft_q15_4096": "cfft_q15",
          "fir_f32": "fir_f32", "fir_q15": "fir_q15", "fir_q31": "fir_q31", "fir_fast_q15": "fir_fast_q15",
          "fir_fast_q31": "fir_fast_q31", "mat_mult_f32": "mat_mult_f32",
          "mfcc_f32": "mfcc_f32", "mat_mult_q15": "mat_mult_q15", "mat_mult_q31": "mat_mult_q31",
          "mat_mult_fast_q31": "mat_mult_fast_q31", "rfft_f32": "rfft_f32", "conv_f32": "conv_f32", "rfft_q31": "rfft_q31", "rfft_q15": "rfft_q15"}[workload]
    nn = 256 if workload.startswith("mat_mult") else n  # 1024^3 takes seconds per matrix on one core
    out = subprocess.run([exe, wl, str(nn), str(threads), str(secs)], capture_output=True, text=True,
                         timeout=120)
    r = json.loads(out.stdout)
    if workload.startswith("mat_mult"):
        return {"value": round(r["gflops"] * 1e-3, 6), "unit": "TFLOP/s" if workload.endswith("f32") else "TOPS",
                "cores": threads, "kind": kind,
                "sample": f"{threads} threads x {secs:.0f} s of arm_{workload} {nn}^3 (reference scalar C)"}
    return {"value": round(r["gsamples_per_s"], 6), "unit": "Gsamples/s", "cores": threads, "kind": kind,
            "sample": f"{threads} threads x {secs:.0f} s, {wl} n={nn}, {int(r['samples'])} samples "
                      f"(reference scalar C, gcc -O2)"}


# ------------------------------------------------------------------ timed loops
def time_launches(launch, steps, warmup, world):
    """W untimed, then K timed launches between barriers; returns (wall s, avg kernel ms)."""
    for s in range(warmup):
        launch(s)
    barrier(world)
    stream = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for s in range(steps):
        evs[s][0].record(stream)
        launch(warmup + s)
        evs[s][1].record(stream)
    barrier(world)
    wall = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    return wall, kern_ms


def run_cfft(kind, n, batch, steps, warmup, world, rank, check=True):
    S = dsp.const_instance(f"arm_cfft_sR_{kind}_len{n}")
    data = synth(kind, batch * 2 * n, rank).view(batch, 2 * n)
    rows = sorted({0, 1, batch // 2, batch - 1})
    before = data[rows].cpu().numpy().copy()
    flags = flag_sequence(warmup + steps)

    def launch(s):
        dsp.cfft_batch(S, data, flags[s], 1)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    parity = None
    if check:
        # replay the exact flag sequence on the sampled rows with the CPU checker
        host, hk = cpu_checker()
        want = before
        for f in flags:
            want = host.cfft_many(kind, n, want, f, 1)
        got = data[rows].cpu().numpy()
        # plus a fresh 64-transform batch through one launch
        fresh = synth(kind, 64 * 2 * n, rank, salt=17).view(64, 2 * n)
        fin = fresh.cpu().numpy()
        dsp.cfft_batch(S, fresh, 0, 1)
        torch.cuda.synchronize()
        fresh_got = fresh.cpu().numpy()
        fresh_want = host.cfft_many(kind, n, fin, 0, 1)
        rec = {"rank": rank,
               "gpu_digest": parallel.digest(np.concatenate([got.ravel(), fresh_got.ravel()]).view(np.uint8)),
               "ref_digest": parallel.digest(np.concatenate([want.ravel(), fresh_want.ravel()]).view(np.uint8))}
        all_ok, combined = parallel.checksum_of_checksums(parallel.gather_objects(WORLD, rec))
        parity = {"checker": hk, "bit_exact": bool(all_ok), "transforms_checked_per_rank": len(rows) + 64,
                  "timed_buffer_rows_replayed": len(rows), "steps_replayed": len(flags),
                  "ranks_checked": world, "checksum_of_checksums": f"{combined:016x}"}
    return wall, kern_ms, parity


def run_fir(kind, taps, batch, steps, warmup, world, rank, block=4096):
    """kind: f32 | q15 | q31 | fast_q15 | fast_q31 (arm_fir_<kind>), full-range fixed point."""
    import ctypes as C
    base = kind[-3:]
    rng = np.random.default_rng(5)
    S = {"f32": dsp.arm_fir_instance_f32, "q15": dsp.arm_fir_instance_q15, "q31": dsp.arm_fir_instance_q31}[base]()
    if base == "f32":
        c = torch.from_numpy((rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)).cuda()
    else:
        bits, dt = (15, np.int16) if base == "q15" else (31, np.int32)
        c = torch.from_numpy(rng.integers(-(1 << bits), 1 << bits, taps).astype(dt)).cuda()
    src = synth(base, batch * block, rank).view(batch, block)
    S.numTaps = taps
    S.pCoeffs = C.cast(c.data_ptr(), S._fields_[2][1])
    dst = torch.empty_like(src)
    hist = torch.zeros((batch, taps - 1), dtype=src.dtype, device="cuda")

    def launch(s):
        dsp.fir_batch(S, src, dst, hist, kind=kind)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    # parity: two filters, one block, from zero history, vs the checker
    host, hk = cpu_checker()
    h0 = torch.zeros((2, taps - 1), dtype=src.dtype, device="cuda")
    d0 = torch.empty((2, block), dtype=src.dtype, device="cuda")
    dsp.fir_batch(S, src[:2].contiguous(), d0, h0, kind=kind)
    torch.cuda.synchronize()
    ok = all(d0[f].cpu().numpy().tobytes() ==
             host.fir(kind, c.cpu().numpy(), [src[f].cpu().numpy()])[0][0].tobytes() for f in range(2))
    return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "filters_checked": 2}


def run_mat(dim, batch, steps, warmup, world, rank):
    a = synth("f32", batch * dim * dim, rank).view(batch, dim, dim) * 2
    b = synth("f32", batch * dim * dim, rank, salt=3).view(batch, dim, dim) * 2
    c = torch.empty_like(a)

    def launch(s):
        dsp.mat_mult_batch(a, b, c)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    exact = (a[0].double() @ b[0].double())
    err = (c[0].double() - exact).abs().max().item()
    bound = float(4 * dim * np.finfo(np.float32).eps * (a[0].double().abs() @ b[0].double().abs()).max().item())
    return wall, kern_ms, {"checker": "float64 GEMM of matrix 0", "max_abs_err": float(err), "bound": bound,
                           "within_bound": bool(err <= bound)}


def run_rfft(n, batch, steps, warmup, world, rank):
    """arm_rfft_fast_f32 forward over [batch][n] real frames -> [batch][n] packed spectra
    (the forward transform also overwrites its input, as in the reference)."""
    S = dsp.const_instance(f"arm_rfft_fast_sR_f32_len{n}")
    p = synth("f32", batch * n, rank).view(batch, n)
    out = torch.empty_like(p)
    def launch(s):
        dsp.rfft_fast_batch(S, p, out, 0)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    host, hk = cpu_checker()
    fresh = synth("f32", 64 * n, rank, salt=41).view(64, n)
    want = np.stack([host.rfft(n, r, 0)[0] for r in fresh.cpu().numpy()])
    fo = torch.empty_like(fresh)
    dsp.rfft_fast_batch(S, fresh.clone(), fo, 0)
    torch.cuda.synchronize()
    ok = fo.cpu().numpy().tobytes() == want.tobytes()
    return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "transforms_checked": 64}


def run_rfft_fixed(kind, n, batch, steps, warmup, world, rank):
    """arm_rfft_q31 / _q15 forward over [batch][n] full-range real signals -> [batch][2n]
    spectra; bit-exact check of 16 fresh signals (spectrum and overwritten input)."""
    S = dsp.arm_rfft_instance_q31() if kind == "q31" else dsp.arm_rfft_instance_q15()
    assert getattr(dsp, f"arm_rfft_init_{kind}")(S, n, 0, 1) == 0
    src = synth(kind, batch * n, rank).view(batch, n)
    out = torch.empty((batch, 2 * n), dtype=src.dtype, device="cuda")

    def launch(s):
        dsp.rfft_fixed_batch(S, src, out)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    host, hk = cpu_checker()
    fresh = synth(kind, 16 * n, rank, salt=43).view(16, n)
    fin = fresh.cpu().numpy()
    fo = torch.empty((16, 2 * n), dtype=src.dtype, device="cuda")
    dsp.rfft_fixed_batch(S, fresh, fo)
    torch.cuda.synchronize()
    want = [host.rfft_fixed(kind, n, fin[r], 0, 1) for r in range(16)]
    ok = (fo.cpu().numpy().tobytes() == np.stack([w[0] for w in want]).tobytes()
          and fresh.cpu().numpy().tobytes() == np.stack([w[1] for w in want]).tobytes())
    return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "signals_checked": 16}


def run_conv(taps, batch, steps, warmup, world, rank, block=4096):
    """arm_conv_f32 of `batch` 4096-sample signals with one shared 128-sample kernel
    (the FIR config's shape): outputs of block + taps - 1 samples."""
    rng = np.random.default_rng(6)
    a = synth("f32", batch * block, rank).view(batch, block)
    b = torch.from_numpy((rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)).cuda()
    out = torch.empty((batch, block + taps - 1), dtype=torch.float32, device="cuda")

    def launch(s):
        dsp.conv_batch(a, b, out)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    host, hk = cpu_checker()
    ok = all(out[i].cpu().numpy().tobytes() == host.conv("f32", a[i].cpu().numpy(), b.cpu().numpy()).tobytes()
             for i in (0, batch - 1))
    return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "items_checked": 2}


def run_mfcc(n, batch, steps, warmup, world, rank):
    import mfcc_cfg
    g = mfcc_cfg.golden()
    cfg = mfcc_cfg.suite_cfg(g, n)
    m = dsp.MfccF32(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
    frames = synth("f32", batch * n, rank).view(batch, n)
    work = torch.empty_like(frames)
    out = torch.empty((batch, m.nb_dct), dtype=torch.float32, device="cuda")

    def launch(s):
        m.batch(frames, out, work)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    host, hk = cpu_checker()
    fresh = synth("f32", 64 * n, rank, salt=29).view(64, n)
    want = host.mfcc(cfg, fresh.cpu().numpy())
    got = m.batch(fresh.clone()).cpu().numpy()
    err = np.abs(got.astype(np.float64) - want)
    return wall, kern_ms, {"checker": hk, "frames_checked": 64, "max_abs_err": float(err.max()),
                           "within_tolerance": bool(np.all(err <= 2e-5 + 1e-6 * np.abs(want))),
                           "bit_exact_fraction": float(np.mean(got.view(np.uint32) == want.view(np.uint32))),
                           "tolerance": "2e-5 + 1e-6*|ref| (device logf vs host libm logf; other stages exact)"}


def run_mat_fixed(kind, dim, batch, steps, warmup, world, rank):
    """arm_mat_mult_q15 / _q31 (byte-sliced i8 MFMA) or _fast_q31 (VALU), full-range operands,
    bit-exact check of matrix 0 against the CPU checker."""
    a = synth(kind[-3:], batch * dim * dim, rank).view(batch, dim, dim)
    b = synth(kind[-3:], batch * dim * dim, rank, salt=3).view(batch, dim, dim)
    c = torch.empty_like(a)
    fast = kind.startswith("fast")

    def launch(s):
        dsp.mat_mult_batch(a, b, c, fast=fast)

    wall, kern_ms = time_launches(launch, steps, warmup, world)
    host, hk = cpu_checker()
    st, want = host.mat_mult_fixed(kind, a[0].cpu().numpy(), b[0].cpu().numpy())
    ok = st == 0 and c[0].cpu().numpy().tobytes() == want.tobytes()
    return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "matrices_checked": 1}


def pmc_traffic(workload):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, when present."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    return json.load(open(p)).get(workload, {}).get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfft_f32_1024", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="items per GPU (default: the BASELINE config)")
    ap.add_argument("--fftlen", type=int, default=0,
                    help="cfft workloads: another fftLen (16..4096), batch scaled to the same bytes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-companion", action="store_true", help="skip the q31 companion measurement")
    ap.add_argument("--dist-backend", default=None, help="nccl (default, RCCL) or gloo (rehearsal)")
    args = ap.parse_args()

    global WORLD
    WORLD = parallel.init(backend=args.dist_backend)
    world, rank = WORLD.size, WORLD.rank
    kind, n, batch0, bps = WORKLOADS[args.workload]
    if args.fftlen and args.workload.startswith(("cfft", "rfft")):   # same bytes per launch
        batch0 = max(1, batch0 * n // args.fftlen)
        n = args.fftlen
    batch = args.batch or batch0
    if args.workload.startswith("cfft"):
        wall, kern_ms, parity = run_cfft(kind, n, batch, args.steps, args.warmup, world, rank)
        units = batch * n                                 # complex samples per launch per GPU
        algo_bytes = units * bps
    elif args.workload.startswith("fir"):
        wall, kern_ms, parity = run_fir(kind[4:], n, batch, args.steps, args.warmup, world, rank)
        units = batch * 4096
        algo_bytes = units * bps + batch * (n - 1) * bps  # in + out + history read/write
    elif args.workload in ("mat_mult_q15", "mat_mult_q31", "mat_mult_fast_q31"):
        wall, kern_ms, parity = run_mat_fixed(kind[3:], n, batch, args.steps, args.warmup, world, rank)
        units = batch
        algo_bytes = None
    elif args.workload == "conv_f32":
        wall, kern_ms, parity = run_conv(n, batch, args.steps, args.warmup, world, rank)
        units = batch * (4096 + n - 1)                     # output samples
        algo_bytes = batch * 4096 * 4 + units * 4          # signal in + output
    elif args.workload == "rfft_f32":
        wall, kern_ms, parity = run_rfft(n, batch, args.steps, args.warmup, world, rank)
        units = batch * n                                  # real input samples
        algo_bytes = units * bps                           # N floats in, N floats out
    elif args.workload in ("rfft_q31", "rfft_q15"):
        wall, kern_ms, parity = run_rfft_fixed(kind[4:], n, batch, args.steps, args.warmup, world, rank)
        units = batch * n                                  # real input samples
        algo_bytes = units * bps                           # N in, N written back, 2N spectrum out
    elif args.workload == "mfcc_f32":
        wall, kern_ms, parity = run_mfcc(n, batch, args.steps, args.warmup, world, rank)
        units = batch * n                                  # input samples
        algo_bytes = units * bps + batch * 13 * 4          # frames in + coefficients out
    else:
        wall, kern_ms, parity = run_mat(n, batch, args.steps, args.warmup, world, rank)
        units = batch                                      # matrices
        algo_bytes = None

    wall = allreduce_max(wall, world)
    kern_ms = allreduce_max(kern_ms, world)
    total_units = units * world * args.steps

    line = {"metric": METRIC, "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "data": "synthetic (per-rank seeded generator, rank-local, no scatter)"}
    if args.workload == "mat_mult_fast_q31":
        ops = 2.0 * n * n * n * batch
        line.update(value=round(total_units * 2.0 * n ** 3 / wall * 1e-12, 4), unit="TOPS (2*M*N*K int MAC)",
                    dtype="q31 (per-product high word, modular q31 accumulator)",
                    config={"workload": f"arm_mat_mult_fast_q31 {n}x{n}x{n} batch={batch}/GPU",
                            "dims": [n, n, n], "batch_per_gpu": batch, "parallelism": f"dp{world} shards"})
        # per MAC: one v_mul_hi_i32 + half a v_add3_u32 (two products summed per add3) = 1.5 lane-instr
        lane_ops = 1.5 * (ops / 2) / (kern_ms * 1e-3) * 1e-12
        line["roofline"] = {"bound": "valu", "achieved": round(lane_ops, 2), "peak": 39.3,
                            "unit": "T VALU lane-instr/s (256 CU x 4 SIMD x 16 lanes x 2.4 GHz)",
                            "frac": round(lane_ops / 39.3, 4), "traffic": None, "avg_kernel_ms": round(kern_ms, 4)}
    elif args.workload in ("mat_mult_q15", "mat_mult_q31"):
        planes = 2 if args.workload.endswith("q15") else 4
        ops = 2.0 * n * n * n * batch
        line.update(value=round(total_units * 2.0 * n ** 3 / wall * 1e-12, 4), unit="TOPS (2*M*N*K int MAC)",
                    dtype=f"{kind[3:]} (exact int64 sums via {planes}x{planes} i8 byte planes)",
                    config={"workload": f"arm_mat_mult_{kind[3:]} {n}x{n}x{n} batch={batch}/GPU",
                            "dims": [n, n, n], "batch_per_gpu": batch, "parallelism": f"dp{world} shards"})
        i8 = ops * planes * planes / (kern_ms * 1e-3) * 1e-12
        line["roofline"] = {"bound": "mfma", "achieved": round(i8, 2), "peak": 5000.0,
                            "unit": "TOPS (i8 MFMA ops incl. the byte-plane products)", "frac": round(i8 / 5000.0, 4),
                            "traffic": None, "avg_kernel_ms": round(kern_ms, 4)}
    elif args.workload == "mat_mult_f32":
        flops = 2.0 * n * n * n * batch
        line.update(value=round(total_units * 2.0 * n ** 3 / wall * 1e-12, 4), unit="TFLOP/s", dtype="f32",
                    config={"workload": f"arm_mat_mult_f32 {n}x{n}x{n} batch={batch}/GPU (BASELINE configs[4])",
                            "dims": [n, n, n], "batch_per_gpu": batch, "parallelism": f"dp{world} shards"})
        achieved = flops / (kern_ms * 1e-3) * 1e-12
        line["roofline"] = {"bound": "mfma", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                            "traffic": pmc_traffic(args.workload), "avg_kernel_ms": round(kern_ms, 4)}
    else:
        line.update(value=round(total_units / wall * 1e-9, 3), unit="Gsamples/s",
                    dtype={"f32": "f32", "q31": "q31 (int32)", "q15": "q15 (int16)", "fir_f32": "f32",
                           "fir_q15": "q15 (int16 x int16 -> int64)", "mfcc": "f32",
                           "fir_q31": "q31 (int32 x int32 -> int64)", "fir_fast_q15": "q15 (int32 wrap accumulator)",
                           "fir_fast_q31": "q31 (rounded high-word accumulator)", "rfft": "f32", "conv": "f32",
                           "rfftq31": "q31 (int32)", "rfftq15": "q15 (int16)"}[kind])
        if args.workload.startswith("cfft"):
            cfg_tag = ("BASELINE configs[1]" if (kind == "f32" and n == 1024) else
                       "BASELINE configs[3]" if (kind != "f32" and n == 4096) else
                       "size sweep, not a BASELINE config")
            line["config"] = {"workload": f"arm_cfft_{kind} N={n} batch={batch}/GPU in place, bitReverseFlag=1, "
                                          f"alternating fwd/inv ({cfg_tag})",
                              "fftLen": n, "batch_per_gpu": batch, "parallelism": f"dp{world} shards"}
        elif kind == "conv":
            line["config"] = {"workload": f"arm_conv_f32 4096 (*) {n} (shared kernel), batch={batch}/GPU",
                              "srcALen": 4096, "srcBLen": n, "batch_per_gpu": batch, "parallelism": f"dp{world} shards"}
        elif kind == "rfft":
            line["config"] = {"workload": f"arm_rfft_fast_f32 N={n} forward, batch={batch}/GPU", "fftLen": n,
                              "batch_per_gpu": batch, "parallelism": f"dp{world} shards"}
        elif kind in ("rfftq31", "rfftq15"):
            line["config"] = {"workload": f"arm_rfft_{kind[4:]} N={n} forward (inner CFFT {n // 2}), "
                                          f"batch={batch}/GPU", "fftLenReal": n, "batch_per_gpu": batch,
                              "parallelism": f"dp{world} shards"}
        elif kind == "mfcc":
            line["config"] = {"workload": f"arm_mfcc_f32 fftLen={n} 20 Mel / 13 DCT (reference MFCC F32 suite "
                                          f"tables) batch={batch} frames/GPU", "fftLen": n, "batch_per_gpu": batch,
                              "parallelism": f"dp{world} shards"}
        else:
            line["config"] = {"workload": f"arm_{kind} numTaps={n} blockSize=4096 batch={batch}/GPU "
                                          + ("(BASELINE configs[2])" if kind == "fir_f32" else "(configs[2] shape, q15)"),
                              "numTaps": n, "blockSize": 4096,
                              "batch_per_gpu": batch, "parallelism": f"dp{world} shards"}
        achieved = algo_bytes / (kern_ms * 1e-3) * 1e-9
        line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(args.workload),
                            "algorithmic_bytes_per_launch": algo_bytes, "avg_kernel_ms": round(kern_ms, 4)}
        if args.workload == "conv_f32":
            valu = units * n * 2 / (kern_ms * 1e-3) * 1e-12
            line["roofline"]["valu_tflops_nofma"] = {"achieved": round(valu, 2), "peak": FP32_NOFMA_TFLOPS,
                                                     "frac": round(valu / FP32_NOFMA_TFLOPS, 4)}
        if args.workload == "rfft_f32":
            # the forward transform also leaves the inner CFFT output in p (reference semantics)
            line["roofline"]["bytes_moved_per_sample"] = 12
        if args.workload == "fir_fast_q15":
            valu = units * n / 2 / (kern_ms * 1e-3) * 1e-12      # one accumulating v_dot2 per tap pair
            line["roofline"]["valu_tops_dot2"] = {"achieved": round(valu, 2), "peak": FP32_NOFMA_TFLOPS,
                                                  "frac": round(valu / FP32_NOFMA_TFLOPS, 4)}
        if args.workload == "fir_q15":
            # one v_dot2_i32_i16 per tap pair per h/l half: T VALU ops per output sample
            valu = units * n / (kern_ms * 1e-3) * 1e-12
            line["roofline"]["valu_tops_dot2"] = {"achieved": round(valu, 2), "peak": FP32_NOFMA_TFLOPS,
                                                  "frac": round(valu / FP32_NOFMA_TFLOPS, 4)}
        if args.workload == "fir_f32":
            valu = units * n * 2 / (kern_ms * 1e-3) * 1e-12
            line["roofline"]["valu_tflops_nofma"] = {"achieved": round(valu, 2), "peak": FP32_NOFMA_TFLOPS,
                                                     "frac": round(valu / FP32_NOFMA_TFLOPS, 4)}
    line["parity"] = parity

    if args.workload == "cfft_f32_1024" and not args.no_companion:
        qb = 1 << 18
        w2, k2, p2 = run_cfft("q31", 4096, qb, args.steps, args.warmup, world, rank)
        w2 = allreduce_max(w2, world)
        k2 = allreduce_max(k2, world)
        ach = qb * 4096 * 16 / (k2 * 1e-3) * 1e-9
        line["companion_q31"] = {"workload": f"arm_cfft_q31 N=4096 batch={qb}/GPU in place, bitReverseFlag=1",
                                 "value": round(qb * 4096 * world * args.steps / w2 * 1e-9, 3), "unit": "Gsamples/s",
                                 "hbm_gbs": round(ach, 1), "hbm_frac": round(ach / HBM_PEAK_GBS, 4),
                                 "avg_kernel_ms": round(k2, 4), "traffic": pmc_traffic("cfft_q31_4096"),
                                 "parity": p2}

    if world == 1 and rank == 0 and not args.no_cpu_baseline:
        try:
            line["cpu_baseline"] = cpu_baseline(args.workload, n)
        except Exception as e:  # a missing/failed baseline must not hide the GPU number
            log("cpu_baseline failed:", e)
            line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    parallel.shutdown(WORLD)


if __name__ == "__main__":
    main()
