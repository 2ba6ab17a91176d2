#!/usr/bin/env python3
"""Benchmark of the MI355X CMSIS-DSP backend — the BASELINE.json headline.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload WL] [--batch B]
                  [--scaling weak|strong] [--global-batch G]

Default line (BASELINE.json metric "Gsamples/sec batched arm_cfft_f32 N=1024 (+ q31
bit-exact) at 1/2/4/8 GPU"):
  * value: configs[1] — batched arm_cfft_f32, fftLen 1024, 2^20 transforms per GPU (8 GiB
    in HBM, in place), bitReverseFlag 1; a step is one pass over the batch, alternating
    forward / inverse; whole-job complex samples per second; weak scaling.
  * config3: configs[3] — arm_cfft_q31 AND arm_cfft_q15, fftLen 4096, ONE global batch of
    2^20 transforms split over the ranks in contiguous slices (strong scaling), each
    bit-exact against the reference scalar C on replayed rows of every rank.
  * roofline of the dominant kernel (HIP-event average launch duration on the launch
    stream), cpu_baseline (the reference scalar C on this host: one core and all cores).

--gpus N > 1 without a torchrun environment: this process starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a CHILD before any
GPU call, forwards its output and exits with its code.  Under torchrun every rank pins
GPU LOCAL_RANK, uses the nccl (RCCL) backend, and times between barriers; MAX over ranks.
Other workloads: see WORKLOADS (--workload).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3     # dense f32 MFMA / packed-FMA VALU peak
FP32_NOFMA_TFLOPS = 78.6     # separate v_mul_f32 + v_add_f32 (bit-exact FIR)
METRIC = "Gsamples/sec batched arm_cfft_f32 N=1024 (+ q31 bit-exact) at 1/2/4/8 GPU"
CONFIG3_GLOBAL_BATCH = 1 << 20   # BASELINE configs[3]: N=4096 batch=1M, sharded
CPU_THREADS_MAX = 16             # the GPU box's CPU share per GPU
SETTLE_MS = 40.0                 # device time of untimed launches before the W warmup steps

WORKLOADS = {
    # name: (kind, fftLen / taps, default batch per GPU, algorithmic bytes per sample)
    "cfft_f32_1024": ("f32", 1024, 1 << 20, 16),
    "cfft_q31_4096": ("q31", 4096, 1 << 18, 16),
    "cfft_q15_4096": ("q15", 4096, 1 << 18, 8),
    "fir_f32": ("fir_f32", 128, 1 << 16, 8),
    "fir_f32_fma": ("fir_f32_fma", 128, 1 << 16, 8),      # opt-in tolerance path (v_fma_f32)
    "fir_q15": ("fir_q15", 128, 1 << 16, 4),
    "fir_q31": ("fir_q31", 128, 1 << 16, 8),
    "fir_fast_q15": ("fir_fast_q15", 128, 1 << 16, 4),
    "fir_fast_q31": ("fir_fast_q31", 128, 1 << 16, 8),
    "mat_mult_f32": ("mat", 1024, 256, None),
    "mfcc_f32": ("mfcc", 1024, 1 << 18, 4),
    # algorithmic bytes per sample: the frame read once (the batched API's d_src is work space,
    # arm_math_mi355x.h), + 13 coefficients per frame -- as mfcc_f32
    "mfcc_q31": ("mfccq31", 1024, 1 << 18, 4),
    "mfcc_q15": ("mfccq15", 1024, 1 << 18, 2),
    "rfft_f32": ("rfft", 1024, 1 << 20, 8),
    # arm_rfft_fast_f32_batch_ex(ARM_MI355X_RFFT_P_SCRATCH): p is scratch, not written back
    "rfft_f32_pscratch": ("rfft", 1024, 1 << 20, 8),
    # real length 8192 (inner CFFT 4096 = the fixed-point specialist); bytes per sample:
    # N words in, N words written back (the inner CFFT overwrites pSrc), 2N words out
    "rfft_q31": ("rfftq31", 8192, 1 << 16, 16),
    "rfft_q15": ("rfftq15", 8192, 1 << 16, 8),
    "conv_f32": ("conv", 128, 1 << 16, 8),
    "mat_mult_q7": ("matq7", 1024, 64, None),
    "mat_mult_q15": ("matq15", 1024, 64, None),
    "mat_mult_q31": ("matq31", 1024, 64, None),
    "mat_mult_fast_q31": ("matfast_q31", 1024, 64, None),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (one per GPU); default 1 or WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfft_f32_1024", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="items per GPU (weak scaling; default: the BASELINE config)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default="weak",
                    help="cfft workloads: strong = one --global-batch split over the ranks")
    ap.add_argument("--global-batch", type=int, default=CONFIG3_GLOBAL_BATCH)
    ap.add_argument("--fftlen", type=int, default=0,
                    help="cfft workloads: another fftLen (16..4096), batch scaled to the same bytes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-config3", "--no-companion", dest="no_config3", action="store_true",
                    help="skip the configs[3] q31 + q15 N=4096 strong-scaling measurement")
    ap.add_argument("--dist-backend", default=None, help="nccl (default on GPUs, RCCL) or gloo (rehearsal)")
    ap.add_argument("--scatter", action="store_true",
                    help="configs[3]: also time rank 0 scattering the global q31 / q15 batch to the ranks "
                         "(point-to-point over RCCL/xGMI), reported beside the compute (SURVEY 8e)")
    ap.add_argument("--cpu-secs", type=float, default=None,
                    help="seconds per CPU-baseline leg (default 1 s all-core, 3 s one core)")
    ap.add_argument("--dry-run", action="store_true",
                    help="plumbing only (CPU, gloo): launch, shard spans, reductions and the line, no device work")
    return ap.parse_args(argv)


# ------------------------------------------------------------------ stdout = the JSON line only
_LINE_FD = None


def reserve_stdout():
    """Point fd 1 at stderr before torch, RCCL or the library load (RCCL prints its version
    banner on fd 1 at init, which a driver running torch.distributed.run directly would read
    beside the line) and keep a duplicate of the original fd 1 for the JSON line alone."""
    global _LINE_FD
    sys.stdout.flush()
    _LINE_FD = os.dup(1)
    os.dup2(2, 1)


def emit_line(line):
    data = json.dumps(line) + "\n"
    if _LINE_FD is None:
        print(data, end="", flush=True)
    else:
        sys.stdout.flush()
        os.write(_LINE_FD, data.encode())


# ------------------------------------------------------------------ N-rank launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args, argv):
    """Start torch.distributed.run as a child (nothing in this process has touched the
    GPU: torch / the library are imported only after this decision), forward its output,
    return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__), *argv]
    log("bench: launching", args.gpus, "ranks:", " ".join(cmd))
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "4")
    # stdout carries only the JSON line: library chatter the ranks print (e.g. gloo's
    # connection messages) is passed on to stderr
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True)
    for line in proc.stdout:
        (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
        sys.stdout.flush()
    return proc.wait()


# ------------------------------------------------------------------ CPU baseline
def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_share():
    """Threads for the all-core leg: the CPUs this process may run on, capped at the box's
    per-GPU share (os.cpu_count() reports the whole machine there)."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count() or 1
    return max(1, min(CPU_THREADS_MAX, avail)), os.cpu_count() or avail


_CPU_WL = {"cfft_f32_1024": "cfft_f32", "cfft_q31_4096": "cfft_q31", "cfft_q15_4096": "cfft_q15",
           "fir_f32": "fir_f32", "fir_f32_fma": "fir_f32", "fir_q15": "fir_q15", "fir_q31": "fir_q31",
           "fir_fast_q15": "fir_fast_q15",
           "fir_fast_q31": "fir_fast_q31", "mat_mult_f32": "mat_mult_f32", "mfcc_f32": "mfcc_f32",
           "mfcc_q31": "mfcc_q31", "mfcc_q15": "mfcc_q15",
           "mat_mult_q7": "mat_mult_q7", "mat_mult_q15": "mat_mult_q15", "mat_mult_q31": "mat_mult_q31", "mat_mult_fast_q31": "mat_mult_fast_q31",
           "rfft_f32": "rfft_f32", "rfft_f32_pscratch": "rfft_f32", "conv_f32": "conv_f32", "rfft_q31": "rfft_q31", "rfft_q15": "rfft_q15"}


def cpu_baseline(workload, n, all_secs=1.0, one_secs=3.0):
    """The reference scalar C (oracle/_ref/bench_ref, else the restatement) on this host:
    one core for `one_secs`, then all the process's cores (<= 16) for `all_secs` each —
    a bounded sample of the same workload (~20 thread-seconds)."""
    exe_ref = os.path.join(ROOT, "oracle", "_ref", "bench_ref")
    exe_port = os.path.join(ROOT, "oracle", "_build", "bench_port")
    exe, kind = (exe_ref, "reference") if os.path.exists(exe_ref) else (exe_port, "port")
    if not os.path.exists(exe):
        return None
    wl = _CPU_WL[workload]
    nn = n                      # mat_mult: the config's 1024^3 (one matrix takes ~4 s on one core)
    threads, machine = cpu_share()

    def run(t, secs):
        out = subprocess.run([exe, wl, str(nn), str(t), str(secs)], capture_output=True, text=True, timeout=300)
        return json.loads(out.stdout)

    one, allc = run(1, one_secs), run(threads, all_secs)
    mat = workload.startswith("mat_mult")
    pick = (lambda r: r["gflops"] * 1e-3) if mat else (lambda r: r["gsamples_per_s"])
    unit = ("TFLOP/s" if workload.endswith("f32") else "TOPS") if mat else "Gsamples/s"
    what = f"arm_{workload} {nn}^3" if mat else f"{wl} n={nn}"
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    return {"value": round(pick(allc), 6), "unit": unit, "cores": threads, "kind": kind,
            "single_core_value": round(pick(one), 6), "threads": threads, "cpu_model": cpu_model(),
            "machine_logical_cpus": machine, "affinity_cpus": affinity,
            "sample": f"{what}: 1 thread x {one_secs:g} s, then {threads} threads x {all_secs:g} s "
                      f"({int(allc['samples'])} samples), each thread its own buffers "
                      f"(reference scalar C, gcc -O2, no FMA)"}


# ------------------------------------------------------------------ everything below runs in a rank
def main_rank(args):
    sys.path.insert(0, os.path.join(ROOT, "cmsis-dsp_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import torch

    from cmsisdsp_amd import parallel

    if args.dry_run:
        world = parallel.init(backend=args.dist_backend or "gloo", device=False)
    else:
        world = parallel.init(backend=args.dist_backend)
    if args.gpus is not None and args.gpus != world.size:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world.size}: launch with "
                         f"`bench.py --gpus N` (it starts the ranks) or torchrun --nproc-per-node {args.gpus}")
    rank = world.rank

    if args.dry_run:
        return dry_run(args, world, parallel)

    import cmsisdsp_amd as dsp

    # ---------------------------------------------------------------- data + checkers
    def synth(kind, n_words, salt=0):
        """Deterministic rank-local input: uniform[-0.5,0.5) f32 or full-range integers."""
        g = torch.Generator(device="cuda")
        g.manual_seed(parallel.seed_for(rank, salt))
        if kind == "f32":
            return torch.rand(n_words, generator=g, device="cuda", dtype=torch.float32) - 0.5
        hi = 1 << {"q31": 31, "q15": 15, "q7": 7}[kind]
        dt = {"q31": torch.int32, "q15": torch.int16, "q7": torch.int8}[kind]
        return torch.randint(-hi, hi, (n_words,), generator=g, device="cuda", dtype=torch.int64).to(dt)

    def synth_global(kind, n, start, count, block=4096):
        """Rows [start, start+count) of a GLOBAL batch whose content depends only on the
        global transform index (one generator per block of `block` transforms), so every
        world size sees the same data; generated on the device, block by block."""
        dt = {"f32": torch.float32, "q31": torch.int32, "q15": torch.int16}[kind]
        out = torch.empty((count, 2 * n), dtype=dt, device="cuda")
        hi = 1 << (31 if kind == "q31" else 15)
        b0, b1 = start // block, (start + count + block - 1) // block
        for b in range(b0, b1):
            lo, up = max(start, b * block), min(start + count, (b + 1) * block)
            g = torch.Generator(device="cuda")
            g.manual_seed(parallel.block_seed(b, salt=n))
            rows = up - b * block                       # generate the block's prefix up to `up`
            if kind == "f32":
                blk = torch.rand((rows, 2 * n), generator=g, device="cuda", dtype=torch.float32) - 0.5
            else:
                blk = torch.randint(-hi, hi, (rows, 2 * n), generator=g, device="cuda", dtype=torch.int64).to(dt)
            out[lo - start:up - start].copy_(blk[lo - b * block:])
            del blk
        return out

    def cpu_checker():
        """The reference scalar C (oracle/_ref) if present, else the restatement (oracle/_build)."""
        import refs
        try:
            return refs.ref_lib(), "reference"
        except (FileNotFoundError, OSError):
            return refs.oracle_lib(), "port"

    def flag_sequence(steps):
        return [s & 1 for s in range(steps)]            # fwd, inv, fwd, ...

    settle = {"launches": 0}

    def time_launches(launch, steps, warmup):
        """Clock settle, W untimed, then K timed launches between barriers; returns (wall s,
        avg kernel ms).  The settle phase repeats the launch until >= SETTLE_MS of device
        time has passed (at most 64 launches): the GPU's power management dips the clock for
        the first ~10-30 ms of a sustained load (kernel traces: the first launch is fast, the
        next few 5-30 % slow, then steady), which W short warmup steps do not cover.  The
        number of settle launches is reported (settle_launches) and every launch, settle
        included, is replayed by the parity check.  The HIP events are recorded on the stream
        the library launches on (torch's current stream)."""
        stream = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s = 0
        e0.record(stream)
        while s < 64:
            launch(s)
            s += 1
            e1.record(stream)
            e1.synchronize()
            if e0.elapsed_time(e1) >= SETTLE_MS:
                break
        settle["launches"] = s
        for w in range(warmup):
            launch(s + w)
        s += warmup
        parallel.barrier(world)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
        t0 = time.perf_counter()
        for k in range(steps):
            evs[k][0].record(stream)
            launch(s + k)
            evs[k][1].record(stream)
        parallel.barrier(world)
        wall = time.perf_counter() - t0
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
        settle["total"] = s + steps
        return wall, kern_ms

    # ---------------------------------------------------------------- workloads
    def run_cfft(kind, n, batch, steps, warmup, strong_span=None):
        """Weak: `batch` rank-local transforms.  Strong: strong_span = (start, count) of the
        global batch.  Parity: the timed buffer's sampled rows replayed through the exact
        flag sequence with the CPU checker, plus a fresh 64-transform launch, on every rank."""
        S = dsp.const_instance(f"arm_cfft_sR_{kind}_len{n}")
        if strong_span is None:
            data = synth(kind, batch * 2 * n).view(batch, 2 * n)
        else:
            data = synth_global(kind, n, *strong_span)
            batch = strong_span[1]
        rows = sorted({0, 1, batch // 2, batch - 1})
        before = data[rows].cpu().numpy().copy()

        def launch(s):
            dsp.cfft_batch(S, data, s & 1, 1)          # fwd, inv, fwd, ...

        wall, kern_ms = time_launches(launch, steps, warmup)
        flags = flag_sequence(settle["total"])
        host, hk = cpu_checker()
        want = before
        for f in flags:
            want = host.cfft_many(kind, n, want, f, 1)
        got = data[rows].cpu().numpy()
        del data
        fresh = synth(kind, 64 * 2 * n, salt=17).view(64, 2 * n)
        fin = fresh.cpu().numpy()
        dsp.cfft_batch(S, fresh, 0, 1)
        torch.cuda.synchronize()
        fresh_got = fresh.cpu().numpy()
        fresh_want = host.cfft_many(kind, n, fin, 0, 1)
        rec = {"rank": rank, "span": list(strong_span) if strong_span else [rank * batch, batch],
               "gpu_digest": parallel.digest(np.concatenate([got.ravel(), fresh_got.ravel()]).view(np.uint8)),
               "ref_digest": parallel.digest(np.concatenate([want.ravel(), fresh_want.ravel()]).view(np.uint8))}
        recs = parallel.gather_objects(world, rec)
        all_ok, combined = parallel.checksum_of_checksums(recs)
        parity = {"checker": hk, "bit_exact": bool(all_ok), "transforms_checked_per_rank": len(rows) + 64,
                  "timed_buffer_rows_replayed": len(rows), "steps_replayed": len(flags),
                  "ranks_checked": len(recs), "per_rank": [{k: r[k] for k in ("rank", "span", "gpu_digest")}
                                                           for r in sorted(recs, key=lambda r: r["rank"])],
                  "checksum_of_checksums": f"{combined:016x}"}
        if strong_span is not None:
            spans = sorted(tuple(r["span"]) for r in recs)
            parity["spans_tile_global_batch"] = bool(
                spans[0][0] == 0 and all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
                and spans[-1][0] + spans[-1][1] == args.global_batch)
        torch.cuda.empty_cache()
        return wall, kern_ms, parity

    def run_fir(kind, taps, batch, steps, warmup, block=4096):
        """kind: f32 | q15 | q31 | fast_q15 | fast_q31 (arm_fir_<kind>), full-range fixed point."""
        import ctypes as C
        base = "f32" if kind == "f32_fma" else kind[-3:]
        rng = np.random.default_rng(5)
        S = {"f32": dsp.arm_fir_instance_f32, "q15": dsp.arm_fir_instance_q15, "q31": dsp.arm_fir_instance_q31}[base]()
        if base == "f32":
            c = torch.from_numpy((rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)).cuda()
        else:
            bits, dt = (15, np.int16) if base == "q15" else (31, np.int32)
            c = torch.from_numpy(rng.integers(-(1 << bits), 1 << bits, taps).astype(dt)).cuda()
        src = synth(base, batch * block).view(batch, block)
        S.numTaps = taps
        S.pCoeffs = C.cast(c.data_ptr(), S._fields_[2][1])
        dst = torch.empty_like(src)
        hist = torch.zeros((batch, taps - 1), dtype=src.dtype, device="cuda")

        def launch(s):
            dsp.fir_batch(S, src, dst, hist, kind=kind)

        wall, kern_ms = time_launches(launch, steps, warmup)
        host, hk = cpu_checker()
        h0 = torch.zeros((2, taps - 1), dtype=src.dtype, device="cuda")
        d0 = torch.empty((2, block), dtype=src.dtype, device="cuda")
        dsp.fir_batch(S, src[:2].contiguous(), d0, h0, kind=kind)
        torch.cuda.synchronize()
        if kind == "f32_fma":       # tolerance: per element vs float64, K 2^-24 sum |x b|
            cc = c.cpu().numpy().astype(np.float64)
            worst = 0.0
            for f in range(2):
                x = np.concatenate([np.zeros(taps - 1), src[f].cpu().numpy().astype(np.float64)])
                w = np.lib.stride_tricks.sliding_window_view(x, taps)
                y64, mag = w @ cc, np.abs(w) @ np.abs(cc)      # pCoeffs are stored time-reversed
                worst = max(worst, float(np.max(np.abs(d0[f].cpu().numpy() - y64) / (taps * 2.0 ** -24 * mag))))
            return wall, kern_ms, {"checker": "float64 FIR", "bit_exact": False, "filters_checked": 2,
                                   "bound": "|y - y64| <= numTaps 2^-24 sum|x b| per element",
                                   "max_err_over_bound": worst, "within_bound": worst <= 1.0}
        ok = all(d0[f].cpu().numpy().tobytes() ==
                 host.fir(kind, c.cpu().numpy(), [src[f].cpu().numpy()])[0][0].tobytes() for f in range(2))
        return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "filters_checked": 2}

    def run_mat(dim, batch, steps, warmup):
        """arm_mat_mult_f32: per-element parity of matrix 0 at full size against float64,
        |C - C64|ij <= K 2^-24 (|A||B|)ij (the recursive-summation bound of an f32 sum, which
        the reference's own sequential sum satisfies); a 16-row slice against the reference
        C itself at 2x that bound; and a negative control: the product of bf16-rounded
        operands must FAIL the same check (so the check can tell f32 from bf16)."""
        a = synth("f32", batch * dim * dim).view(batch, dim, dim) * 2
        b = synth("f32", batch * dim * dim, salt=3).view(batch, dim, dim) * 2
        c = torch.empty_like(a)

        def launch(s):
            dsp.mat_mult_batch(a, b, c)

        wall, kern_ms = time_launches(launch, steps, warmup)
        return wall, kern_ms, mat_parity(a[0], b[0], c[0])

    def mat_parity(a, b, c):
        """Tolerance vs float64 (elementwise K 2^-24 (|A||B|)ij, and rms <= sqrt(K) 2^-24 -- the
        statistic a TF32-class regression fails), 2x that vs the reference's own C on 16 rows,
        and the kernel's stated semantics bit for bit: the k-ordered fmaf chain
        (oracle_mat_mult_f32_fmaf) on the same 16 rows.  Negative controls: bf16- and
        TF32-rounded operands must fail."""
        import refs
        k = a.shape[1]
        a64, b64 = a.double(), b.double()
        exact = a64 @ b64
        mag = a64.abs() @ b64.abs()
        bound = k * 2.0 ** -24 * mag
        err = (c.double() - exact).abs()
        ratio = (err / bound).max().item()
        rms = lambda e: ((e / mag).pow(2).mean().sqrt() / (k ** 0.5 * 2.0 ** -24)).item()
        bf = (a.bfloat16().double() @ b.bfloat16().double())
        bf_over = ((bf - exact).abs() > bound).double().mean().item()
        tf32 = lambda x: ((x.contiguous().view(torch.int32).long() + 0xFFF + ((x.contiguous().view(torch.int32).long() >> 13) & 1))
                          & ~0x1FFF).to(torch.int32).view(torch.float32)
        tf_rms = rms((tf32(a).double() @ tf32(b).double() - exact).abs())
        host, hk = cpu_checker()
        rows = 16
        st, ref = host.mat_mult(a[:rows].cpu().numpy(), b.cpu().numpy())
        ref = torch.from_numpy(ref).double()
        ratio_ref = ((c[:rows].double().cpu() - ref).abs() / (2 * bound[:rows].cpu())).max().item()
        try:
            _, fm = refs.oracle_lib().mat_mult_fmaf(a[:rows].cpu().numpy(), b.cpu().numpy())
            fmaf_exact = bool(c[:rows].cpu().numpy().tobytes() == fm.tobytes())
        except (FileNotFoundError, OSError):
            fmaf_exact = None
        return {"checker": f"float64 GEMM (all of matrix 0) + {hk} arm_mat_mult_f32 ({rows} x {k} x {c.shape[1]})"
                           f" + oracle_mat_mult_f32_fmaf ({rows} rows)",
                "bound": "|C-C64|ij <= K*2^-24*(|A||B|)ij; rms(|C-C64|/(|A||B|)) <= sqrt(K)*2^-24; vs reference: 2x",
                "max_err_over_bound": ratio, "within_bound": bool(ratio <= 1.0),
                "rms_over_bound": rms(err), "max_err_over_bound_vs_reference": ratio_ref,
                "within_bound_vs_reference": bool(ratio_ref <= 1.0),
                "fmaf_chain_bit_exact": fmaf_exact,
                "negative_control_bf16_fraction_rejected": bf_over,
                "negative_control_tf32_rms_over_bound": tf_rms,
                "negative_control_rejected": bool(bf_over > 0.0 and tf_rms > 1.0)}

    def run_rfft(n, batch, steps, warmup, p_scratch=False):
        """arm_rfft_fast_f32 forward over [batch][n] real frames -> [batch][n] packed spectra.
        Default: the forward also overwrites its input with the inner CFFT's output, as the
        reference does, and the parity checks out AND p.  p_scratch: arm_rfft_fast_f32_batch_ex
        with ARM_MI355X_RFFT_P_SCRATCH (p is scratch: not written back), parity on out."""
        S = dsp.const_instance(f"arm_rfft_fast_sR_f32_len{n}")
        p = synth("f32", batch * n).view(batch, n)
        out = torch.empty_like(p)

        def launch(s):
            dsp.rfft_fast_batch(S, p, out, 0, p_scratch=p_scratch)

        wall, kern_ms = time_launches(launch, steps, warmup)
        host, hk = cpu_checker()
        fresh = synth("f32", 64 * n, salt=41).view(64, n)
        refs_ = [host.rfft(n, r, 0) for r in fresh.cpu().numpy()]
        want = np.stack([r[0] for r in refs_])
        want_p = np.stack([r[1] for r in refs_])
        fo, fp = torch.empty_like(fresh), fresh.clone()
        dsp.rfft_fast_batch(S, fp, fo, 0, p_scratch=p_scratch)
        torch.cuda.synchronize()
        ok = fo.cpu().numpy().tobytes() == want.tobytes()
        rec = {"checker": hk, "bit_exact": bool(ok), "transforms_checked": 64}
        if p_scratch:
            rec["p"] = "scratch (ARM_MI355X_RFFT_P_SCRATCH): not compared"
        else:
            rec["p_bit_exact"] = bool(fp.cpu().numpy().tobytes() == want_p.tobytes())
            rec["bit_exact"] = bool(ok and rec["p_bit_exact"])
        return wall, kern_ms, rec

    def run_rfft_fixed(kind, n, batch, steps, warmup):
        """arm_rfft_q31 / _q15 forward over [batch][n] full-range real signals -> [batch][2n]
        spectra; bit-exact check of 16 fresh signals (spectrum and overwritten input)."""
        S = dsp.arm_rfft_instance_q31() if kind == "q31" else dsp.arm_rfft_instance_q15()
        assert getattr(dsp, f"arm_rfft_init_{kind}")(S, n, 0, 1) == 0
        src = synth(kind, batch * n).view(batch, n)
        out = torch.empty((batch, 2 * n), dtype=src.dtype, device="cuda")

        def launch(s):
            dsp.rfft_fixed_batch(S, src, out)

        wall, kern_ms = time_launches(launch, steps, warmup)
        host, hk = cpu_checker()
        fresh = synth(kind, 16 * n, salt=43).view(16, n)
        fin = fresh.cpu().numpy()
        fo = torch.empty((16, 2 * n), dtype=src.dtype, device="cuda")
        dsp.rfft_fixed_batch(S, fresh, fo)
        torch.cuda.synchronize()
        want = [host.rfft_fixed(kind, n, fin[r], 0, 1) for r in range(16)]
        ok = (fo.cpu().numpy().tobytes() == np.stack([w[0] for w in want]).tobytes()
              and fresh.cpu().numpy().tobytes() == np.stack([w[1] for w in want]).tobytes())
        return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "signals_checked": 16}

    def run_conv(taps, batch, steps, warmup, block=4096):
        """arm_conv_f32 of `batch` 4096-sample signals with one shared 128-sample kernel
        (the FIR config's shape): outputs of block + taps - 1 samples."""
        rng = np.random.default_rng(6)
        a = synth("f32", batch * block).view(batch, block)
        b = torch.from_numpy((rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)).cuda()
        out = torch.empty((batch, block + taps - 1), dtype=torch.float32, device="cuda")

        def launch(s):
            dsp.conv_batch(a, b, out)

        wall, kern_ms = time_launches(launch, steps, warmup)
        host, hk = cpu_checker()
        ok = all(out[i].cpu().numpy().tobytes() == host.conv("f32", a[i].cpu().numpy(), b.cpu().numpy()).tobytes()
                 for i in (0, batch - 1))
        return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "items_checked": 2}

    def run_mfcc(n, batch, steps, warmup):
        import mfcc_cfg
        g = mfcc_cfg.golden()
        cfg = mfcc_cfg.suite_cfg(g, n)
        m = dsp.MfccF32(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"], cfg["window"])
        frames = synth("f32", batch * n).view(batch, n)
        work = torch.empty_like(frames)
        out = torch.empty((batch, m.nb_dct), dtype=torch.float32, device="cuda")

        def launch(s):
            m.batch(frames, out, work)

        wall, kern_ms = time_launches(launch, steps, warmup)
        host, hk = cpu_checker()
        fresh = synth("f32", 64 * n, salt=29).view(64, n)
        want = host.mfcc(cfg, fresh.cpu().numpy())
        got = m.batch(fresh.clone()).cpu().numpy()
        err = float(np.nanmax(np.abs(got.astype(np.float64) - want)))
        try:
            libm_ok, libm_bad, glibc = mfcc_cfg.host_libm_status()
        except OSError:
            libm_ok, libm_bad, glibc = None, None, None
        return wall, kern_ms, {"checker": hk, "frames_checked": 64, "bit_exact": got.tobytes() == want.tobytes(),
                               "max_abs_err": err,
                               "within_suite_tolerance": bool(np.all(np.abs(got - want) <= 1e-5 + 1.2e-3 * np.abs(want))),
                               "logf": "host glibc logf restated on the device (host_logf.hpp)",
                               "host_libm": glibc, "host_logf_equals_restated": libm_ok,
                               "host_logf_sampled_mismatches": libm_bad}

    def run_mfcc_fixed(t, n, batch, steps, warmup):
        """arm_mfcc_q31 / _q15 (pre + RFFT + post) on the suite's 1024 tables over full-range
        frames (the pre pass rewrites them in place, as the reference does, so later steps
        process the previous step's windowed frames: the same work per step); 64 fresh frames
        checked bit-exact against the CPU checker."""
        import importlib
        tq = importlib.import_module(f"test_mfcc_{t}")
        g = tq.golden()
        cfg = tq.suite_cfg(g, n)
        m = (dsp.MfccQ31 if t == "q31" else dsp.MfccQ15)(n, cfg["dct"], cfg["pos"], cfg["len"], cfg["coefs"],
                                                         cfg["window"])
        frames = synth(t, batch * n).view(batch, n)
        work = torch.empty((batch, 2 * n), dtype=frames.dtype, device="cuda")
        out = torch.empty((batch, m.nb_dct), dtype=frames.dtype, device="cuda")

        def launch(s):
            m.batch(frames, out, work)

        wall, kern_ms = time_launches(launch, steps, warmup)
        host, hk = cpu_checker()
        fresh = synth(t, 64 * n, salt=31).view(64, n)
        want = getattr(host, f"mfcc_{t}")(cfg, fresh.cpu().numpy())
        got = m.batch(fresh.clone()).cpu().numpy()
        return wall, kern_ms, {"checker": hk, "frames_checked": 64, "bit_exact": bool(got.tobytes() == want.tobytes())}

    def run_mat_fixed(kind, dim, batch, steps, warmup):
        """arm_mat_mult_q7 (one i8 MFMA plane), _q15 / _q31 (byte-sliced i8 MFMA) or _fast_q31 (VALU),
        full-range operands, bit-exact check of matrix 0 against the CPU checker."""
        base = "q7" if kind == "q7" else kind[-3:]
        a = synth(base, batch * dim * dim).view(batch, dim, dim)
        b = synth(base, batch * dim * dim, salt=3).view(batch, dim, dim)
        c = torch.empty_like(a)
        fast = kind.startswith("fast")

        def launch(s):
            dsp.mat_mult_batch(a, b, c, fast=fast)

        wall, kern_ms = time_launches(launch, steps, warmup)
        host, hk = cpu_checker()
        if kind == "q7":
            # the reference's q7 body keeps its output row offset in a uint16_t (arm_mat_mult_q7.c:704,
            # :782): at 1024 x 1024 it overwrites earlier rows.  Check matrix 0 against the exact
            # formula, and the reference on the 64 rows whose offset does not wrap.
            a0, b0 = a[0].cpu().numpy(), b[0].cpu().numpy()
            exact = np.clip(np.matmul(a0.astype(np.int64), b0.astype(np.int64)) >> 7, -128, 127).astype(np.int8)
            got = c[0].cpu().numpy()
            rows = 65536 // dim
            st, want = host.mat_mult_fixed(kind, a0[:rows], b0)
            ok_exact = got.tobytes() == exact.tobytes()
            ok_ref = st == 0 and got[:rows].tobytes() == want.tobytes()
            return wall, kern_ms, {"checker": f"exact int64 formula (all of matrix 0) + {hk} ({rows} rows)",
                                   "bit_exact": bool(ok_exact and ok_ref), "matrices_checked": 1,
                                   "reference_rows_checked": rows}
        st, want = host.mat_mult_fixed(kind, a[0].cpu().numpy(), b[0].cpu().numpy())
        ok = st == 0 and c[0].cpu().numpy().tobytes() == want.tobytes()
        return wall, kern_ms, {"checker": hk, "bit_exact": bool(ok), "matrices_checked": 1}

    def run_scatter(kind, n):
        """SURVEY 8e's separately timed scatter: rank 0 generates the whole configs[3] global
        batch on its GPU and sends every rank its contiguous slice point to point (RCCL over
        xGMI with nccl; CPU tensors with gloo), bracketed by barrier + synchronize; every rank
        then checks its received slice against its own rank-local generation of the same rows."""
        G = args.global_batch
        spans = [parallel.shard(G, r, world_n) for r in range(world_n)]
        esz = 4 if kind == "q31" else 2
        dev = world.backend != "gloo"
        full = synth_global(kind, n, 0, G) if rank == 0 else None
        if rank == 0 and not dev:
            full = full.cpu()
        dt = torch.int32 if kind == "q31" else torch.int16
        out = torch.empty((spans[rank][1], 2 * n), dtype=dt, device="cuda" if dev else "cpu")
        parallel.barrier(world)
        t0 = time.perf_counter()
        parallel.scatter_rows(world, full, spans, out)
        parallel.barrier(world)
        secs = parallel.reduce_max(world, time.perf_counter() - t0)
        ok = bool(torch.equal(out.to("cuda"), synth_global(kind, n, *spans[rank])))
        oks = parallel.gather_objects(world, ok)
        del full, out
        torch.cuda.empty_cache()
        moved = (G - spans[0][1]) * 2 * n * esz              # bytes that left rank 0
        return {"bytes_moved": moved, "ms": round(secs * 1e3, 3),
                "GB_per_s": round(moved / secs * 1e-9, 2) if moved else None,
                "path": "rank 0 -> ranks, point-to-point " + ("RCCL over xGMI (device tensors)" if dev else
                                                             "gloo (host tensors, rehearsal)"),
                "slices_verified": bool(all(oks)), "ranks": world_n,
                "note": "timed separately; never part of value (rank-local generation is the headline)"}

    # ---------------------------------------------------------------- dispatch
    world_n = world.size
    kind, n, batch0, bps = WORKLOADS[args.workload]
    if args.fftlen and args.workload.startswith(("cfft", "rfft")):   # same bytes per launch
        batch0 = max(1, batch0 * n // args.fftlen)
        n = args.fftlen
    batch = args.batch or batch0
    scaling = "weak"
    if args.workload.startswith("cfft"):
        span = None
        if args.scaling == "strong":
            span = parallel.shard(args.global_batch, rank, world_n)
            scaling = "strong"
        wall, kern_ms, parity = run_cfft(kind, n, batch, args.steps, args.warmup, strong_span=span)
        if span is not None:
            batch = max(r["span"][1] for r in parity["per_rank"])   # the largest slice sets the time
        units = batch * n                                 # complex samples per launch per GPU
        algo_bytes = units * bps
    elif args.workload.startswith("fir"):
        wall, kern_ms, parity = run_fir(kind[4:], n, batch, args.steps, args.warmup)
        units = batch * 4096
        algo_bytes = units * bps + batch * (n - 1) * bps  # in + out + history read/write
    elif args.workload in ("mat_mult_q7", "mat_mult_q15", "mat_mult_q31", "mat_mult_fast_q31"):
        wall, kern_ms, parity = run_mat_fixed(kind[3:], n, batch, args.steps, args.warmup)
        units = batch
        algo_bytes = None
    elif args.workload == "conv_f32":
        wall, kern_ms, parity = run_conv(n, batch, args.steps, args.warmup)
        units = batch * (4096 + n - 1)                     # output samples
        algo_bytes = batch * 4096 * 4 + units * 4          # signal in + output
    elif args.workload in ("rfft_f32", "rfft_f32_pscratch"):
        wall, kern_ms, parity = run_rfft(n, batch, args.steps, args.warmup, p_scratch=args.workload.endswith("pscratch"))
        units = batch * n                                  # real input samples
        algo_bytes = units * bps                           # N floats in, N floats out
    elif args.workload in ("rfft_q31", "rfft_q15"):
        wall, kern_ms, parity = run_rfft_fixed(kind[4:], n, batch, args.steps, args.warmup)
        units = batch * n                                  # real input samples
        algo_bytes = units * bps                           # N in, N written back, 2N spectrum out
    elif args.workload == "mfcc_f32":
        wall, kern_ms, parity = run_mfcc(n, batch, args.steps, args.warmup)
        units = batch * n                                  # input samples
        algo_bytes = units * bps + batch * 13 * 4          # frames in + coefficients out
    elif args.workload in ("mfcc_q31", "mfcc_q15"):
        wall, kern_ms, parity = run_mfcc_fixed(args.workload[-3:], n, batch, args.steps, args.warmup)
        units = batch * n                                  # input samples
        algo_bytes = units * bps + batch * 13 * bps        # frames in + coefficients out
    else:
        wall, kern_ms, parity = run_mat(n, batch, args.steps, args.warmup)
        units = batch                                      # matrices
        algo_bytes = None

    wall = parallel.reduce_max(world, wall)
    kern_ms = parallel.reduce_max(world, kern_ms)
    total_units = (args.global_batch * n if scaling == "strong" else units * world_n) * args.steps
    devices = len(set(parallel.gather_objects(world, torch.cuda.current_device())))

    line = {"metric": METRIC, "n_gpus": world_n, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 4), "higher_is_better": True, "scaling": scaling,
            "vs_baseline": None, "data": "synthetic (device generator seeded per rank / per global block; no scatter)",
            "ranks": world_n, "devices_used": devices, "dist_backend": world.backend,
            "settle_launches": settle["launches"], "library": dsp.version()}
    if args.workload == "mat_mult_fast_q31":
        ops = 2.0 * n * n * n * batch
        line.update(value=round(total_units * 2.0 * n ** 3 / wall * 1e-12, 4), unit="TOPS (2*M*N*K int MAC)",
                    dtype="q31 (per-product high word, modular q31 accumulator)",
                    config={"workload": f"arm_mat_mult_fast_q31 {n}x{n}x{n} batch={batch}/GPU",
                            "dims": [n, n, n], "batch_per_gpu": batch, "parallelism": f"dp{world_n} shards"})
        # per MAC: one v_mul_hi_i32 + half a v_add3_u32 (two products summed per add3) = 1.5 lane-instr
        lane_ops = 1.5 * (ops / 2) / (kern_ms * 1e-3) * 1e-12
        line["roofline"] = {"bound": "valu", "achieved": round(lane_ops, 2), "peak": 39.3,
                            "unit": "T VALU lane-instr/s (256 CU x 4 SIMD x 16 lanes x 2.4 GHz)",
                            "frac": round(lane_ops / 39.3, 4), "traffic": None, "avg_kernel_ms": round(kern_ms, 4)}
        vi = valu_issue(args.workload, batch, kern_ms)
        if vi:
            line["roofline"]["valu_issue"] = vi
    elif args.workload == "mat_mult_q7":
        ops = 2.0 * n * n * n * batch
        line.update(value=round(total_units * 2.0 * n ** 3 / wall * 1e-12, 4), unit="TOPS (2*M*N*K int MAC)",
                    dtype="q7 (int8 x int8 -> int32, one i8 MFMA plane)",
                    config={"workload": f"arm_mat_mult_q7 {n}x{n}x{n} batch={batch}/GPU",
                            "dims": [n, n, n], "batch_per_gpu": batch, "parallelism": f"dp{world_n} shards"})
        i8 = ops / (kern_ms * 1e-3) * 1e-12
        hbm = 3.0 * n * n * batch / (kern_ms * 1e-3) * 1e-9       # A, B read once, C written once
        line["roofline"] = {"bound": "mfma", "achieved": round(i8, 2), "peak": 5000.0,
                            "unit": "TOPS (i8 MFMA, dense)", "frac": round(i8 / 5000.0, 4),
                            "traffic": pmc_traffic(args.workload, batch), "avg_kernel_ms": round(kern_ms, 4),
                            "mfma_busy": pmc_field(args.workload, "mfma_busy_frac", batch),
                            "hbm_algorithmic": {"achieved": round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                                "frac": round(hbm / HBM_PEAK_GBS, 4),
                                                "bytes_per_matrix": 3 * n * n}}
    elif args.workload in ("mat_mult_q15", "mat_mult_q31"):
        planes = 2 if args.workload.endswith("q15") else 4
        ops = 2.0 * n * n * n * batch
        line.update(value=round(total_units * 2.0 * n ** 3 / wall * 1e-12, 4), unit="TOPS (2*M*N*K int MAC)",
                    dtype=f"{kind[3:]} (exact int64 sums via {planes}x{planes} i8 byte planes)",
                    config={"workload": f"arm_mat_mult_{kind[3:]} {n}x{n}x{n} batch={batch}/GPU",
                            "dims": [n, n, n], "batch_per_gpu": batch, "parallelism": f"dp{world_n} shards"})
        i8 = ops * planes * planes / (kern_ms * 1e-3) * 1e-12
        line["roofline"] = {"bound": "mfma", "achieved": round(i8, 2), "peak": 5000.0,
                            "unit": "TOPS (i8 MFMA ops incl. the byte-plane products)", "frac": round(i8 / 5000.0, 4),
                            "traffic": None, "avg_kernel_ms": round(kern_ms, 4)}
    elif args.workload == "mat_mult_f32":
        flops = 2.0 * n * n * n * batch
        line.update(value=round(total_units * 2.0 * n ** 3 / wall * 1e-12, 4), unit="TFLOP/s", dtype="f32",
                    config={"workload": f"arm_mat_mult_f32 {n}x{n}x{n} batch={batch}/GPU (BASELINE configs[4])",
                            "dims": [n, n, n], "batch_per_gpu": batch, "parallelism": f"dp{world_n} shards"})
        achieved = flops / (kern_ms * 1e-3) * 1e-12
        line["roofline"] = {"bound": "mfma", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
                            "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                            "traffic": pmc_traffic(args.workload, batch), "avg_kernel_ms": round(kern_ms, 4),
                            "mfma_busy": pmc_field(args.workload, "mfma_busy_frac", batch)}
    else:
        line.update(value=round(total_units / wall * 1e-9, 3), unit="Gsamples/s",
                    dtype={"f32": "f32", "q31": "q31 (int32)", "q15": "q15 (int16)", "fir_f32": "f32",
                           "fir_q15": "q15 (int16 x int16 -> int64)", "mfcc": "f32",
                           "fir_f32_fma": "f32 (fused multiply-add, tolerance)",
                           "fir_q31": "q31 (int32 x int32 -> int64)", "fir_fast_q15": "q15 (int32 wrap accumulator)",
                           "fir_fast_q31": "q31 (rounded high-word accumulator)", "rfft": "f32", "conv": "f32",
                           "rfftq31": "q31 (int32)", "rfftq15": "q15 (int16)", "mfccq31": "q31 (int32)",
                           "mfccq15": "q15 (int16)"}[kind])
        if args.workload.startswith("cfft"):
            cfg_tag = ("BASELINE configs[1]" if (kind == "f32" and n == 1024) else
                       "BASELINE configs[3]" if (kind != "f32" and n == 4096) else
                       "size sweep, not a BASELINE config")
            if scaling == "strong":
                line["config"] = {"workload": f"arm_cfft_{kind} N={n} global batch={args.global_batch} split over "
                                              f"{world_n} ranks, in place, bitReverseFlag=1, alternating fwd/inv "
                                              f"({cfg_tag})", "fftLen": n, "global_batch": args.global_batch,
                                  "parallelism": f"dp{world_n} contiguous slices"}
            else:
                line["config"] = {"workload": f"arm_cfft_{kind} N={n} batch={batch}/GPU in place, bitReverseFlag=1, "
                                              f"alternating fwd/inv ({cfg_tag})",
                                  "fftLen": n, "batch_per_gpu": batch, "parallelism": f"dp{world_n} shards"}
        elif kind == "conv":
            line["config"] = {"workload": f"arm_conv_f32 4096 (*) {n} (shared kernel), batch={batch}/GPU",
                              "srcALen": 4096, "srcBLen": n, "batch_per_gpu": batch,
                              "parallelism": f"dp{world_n} shards"}
        elif kind == "rfft":
            line["config"] = {"workload": f"arm_rfft_fast_f32 N={n} forward, batch={batch}/GPU"
                                          + (", p as scratch (arm_rfft_fast_f32_batch_ex, ARM_MI355X_RFFT_P_SCRATCH)"
                                             if args.workload.endswith("pscratch") else ""), "fftLen": n,
                              "batch_per_gpu": batch, "parallelism": f"dp{world_n} shards"}
        elif kind in ("rfftq31", "rfftq15"):
            line["config"] = {"workload": f"arm_rfft_{kind[4:]} N={n} forward (inner CFFT {n // 2}), "
                                          f"batch={batch}/GPU", "fftLenReal": n, "batch_per_gpu": batch,
                              "parallelism": f"dp{world_n} shards"}
        elif kind in ("mfccq31", "mfccq15"):
            line["config"] = {"workload": f"arm_mfcc_{kind[4:]} fftLen={n} 20 Mel / 13 DCT (reference MFCC "
                                          f"{kind[4:].upper()} suite "
                                          f"tables) batch={batch} frames/GPU", "fftLen": n, "batch_per_gpu": batch,
                              "parallelism": f"dp{world_n} shards"}
        elif kind == "mfcc":
            line["config"] = {"workload": f"arm_mfcc_f32 fftLen={n} 20 Mel / 13 DCT (reference MFCC F32 suite "
                                          f"tables) batch={batch} frames/GPU", "fftLen": n, "batch_per_gpu": batch,
                              "parallelism": f"dp{world_n} shards"}
        else:
            line["config"] = {"workload": f"arm_{kind} numTaps={n} blockSize=4096 batch={batch}/GPU "
                                          + ("(BASELINE configs[2])" if kind == "fir_f32" else "(configs[2] shape)"),
                              "numTaps": n, "blockSize": 4096,
                              "batch_per_gpu": batch, "parallelism": f"dp{world_n} shards"}
        achieved = algo_bytes / (kern_ms * 1e-3) * 1e-9
        prof = (f"{args.workload}_strong{args.global_batch >> 20}M" if scaling == "strong" and args.global_batch % (1 << 20) == 0
                else args.workload if not args.fftlen else f"cfft_{kind}_{n}")
        line["roofline"] = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(prof, batch),
                            "algorithmic_bytes_per_launch": algo_bytes, "avg_kernel_ms": round(kern_ms, 4)}
        if args.workload == "conv_f32":
            valu = units * n * 2 / (kern_ms * 1e-3) * 1e-12
            line["roofline"]["valu_tflops_nofma"] = {"achieved": round(valu, 2), "peak": FP32_NOFMA_TFLOPS,
                                                     "frac": round(valu / FP32_NOFMA_TFLOPS, 4)}
        if args.workload == "rfft_f32":
            # the forward transform also leaves the inner CFFT output in p (reference semantics)
            line["roofline"]["bytes_moved_per_sample"] = 12
        if args.workload == "rfft_f32_pscratch":
            line["roofline"]["bytes_moved_per_sample"] = 8
        if args.workload in ("fir_q15", "fir_fast_q15"):
            # fir_mfma.hip: per 1024 outputs 6 i8 plane products of a 32 x 32 x (32 KS) MFMA tile, KS =
            # ceil((numTaps + 32) / 32): the i8 MFMA work the kernel issues against the 5 POPS dense peak
            # (arm_fir_fast_q15 runs the same kernel with the modular epilogue)
            ks = (n + 32 + 31) // 32
            i8 = units / 1024 * 6 * 2 * 32 * 32 * 32 * ks / (kern_ms * 1e-3) * 1e-12
            line["roofline"]["mfma_i8"] = {"achieved": round(i8, 2), "peak": 5000.0, "unit": "TOPS (i8 MFMA issued)",
                                           "frac": round(i8 / 5000.0, 4), "k_steps": ks, "plane_products": 6}
        if args.workload == "fir_q31":
            # fir_mfma.hip: 16 i8 plane products (4 sample x 4 tap planes) per K step, KS = ceil((numTaps + 31) / 32)
            ks = (n + 31 + 31) // 32
            i8 = units / 1024 * 16 * 2 * 32 * 32 * 32 * ks / (kern_ms * 1e-3) * 1e-12
            line["roofline"]["mfma_i8"] = {"achieved": round(i8, 2), "peak": 5000.0, "unit": "TOPS (i8 MFMA issued)",
                                           "frac": round(i8 / 5000.0, 4), "k_steps": ks, "plane_products": 16}
        if args.workload in ("fir_q15", "fir_q31", "fir_fast_q15", "fir_fast_q31", "mfcc_q31", "mfcc_q15"):
            vi = valu_issue(prof, batch, kern_ms)
            if vi:
                line["roofline"]["valu_issue"] = vi
        if args.workload == "fir_f32":
            valu = units * n * 2 / (kern_ms * 1e-3) * 1e-12
            line["roofline"]["valu_tflops_nofma"] = {"achieved": round(valu, 2), "peak": FP32_NOFMA_TFLOPS,
                                                     "frac": round(valu / FP32_NOFMA_TFLOPS, 4)}
        if args.workload == "fir_f32_fma":
            # SURVEY 8d's FP32-VALU ceiling: 157.3 TFLOP/s / 256 flop per sample = 614 Gsamples/s
            gs = units / (kern_ms * 1e-3) * 1e-9
            line["roofline"]["valu_fp32"] = {"achieved_gsamples": round(gs, 1), "peak_gsamples": 614.0,
                                             "frac": round(gs / 614.0, 4),
                                             "note": "157.3 TFLOP/s FP32 VALU / (2 flop x 128 taps)"}
    line["parity"] = parity

    # ---------------------------------------------------------------- configs[3]
    if args.workload == "cfft_f32_1024" and not args.no_config3:
        torch.cuda.empty_cache()
        span = parallel.shard(args.global_batch, rank, world_n)
        c3 = {"workload": f"arm_cfft_q31 + arm_cfft_q15 N=4096, global batch={args.global_batch} split over "
                          f"{world_n} ranks in contiguous slices, in place, bitReverseFlag=1, alternating fwd/inv "
                          f"(BASELINE configs[3])", "scaling": "strong", "global_batch": args.global_batch}
        for qk, qbps in (("q31", 16), ("q15", 8)):
            w2, k2, p2 = run_cfft(qk, 4096, 0, args.steps, args.warmup, strong_span=span)
            w2 = parallel.reduce_max(world, w2)
            k2 = parallel.reduce_max(world, k2)
            biggest = max(r["span"][1] for r in p2["per_rank"])
            ach = biggest * 4096 * qbps / (k2 * 1e-3) * 1e-9
            c3[qk] = {"value": round(args.global_batch * 4096 * args.steps / w2 * 1e-9, 3), "unit": "Gsamples/s",
                      "settle_launches": settle["launches"],
                      "ms_per_step": round(w2 / args.steps * 1e3, 4), "dtype": "q31 (int32)" if qk == "q31" else
                      "q15 (int16)", "roofline": {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                                                  "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                                                  "traffic": pmc_traffic(f"cfft_{qk}_4096_strong1M", biggest)
                                                  if args.global_batch == 1 << 20 else None,
                                                  "algorithmic_bytes_per_launch": biggest * 4096 * qbps,
                                                  "avg_kernel_ms": round(k2, 4)},
                      "parity": p2}
            if args.global_batch == 1 << 20:
                vi = valu_issue(f"cfft_{qk}_4096_strong1M", biggest, k2)
                if vi:
                    c3[qk]["roofline"]["valu_issue"] = vi
        if args.scatter:
            for qk in ("q31", "q15"):
                c3[qk]["scatter"] = run_scatter(qk, 4096)
        line["config3"] = c3

    if rank == 0 and not args.no_cpu_baseline:
        secs = (args.cpu_secs, args.cpu_secs) if args.cpu_secs else (1.0, 3.0)
        try:
            line["cpu_baseline"] = cpu_baseline(args.workload, n, *secs)
            if "config3" in line:
                for qk in ("q31", "q15"):
                    line["config3"][qk]["cpu_baseline"] = cpu_baseline(f"cfft_{qk}_4096", 4096, secs[0],
                                                                       min(secs[1], 2.0))
            if line["cpu_baseline"] is not None:
                line["cpu_baseline"]["scope"] = (
                    "rank 0's host CPU share (the box allots 16 CPUs per GPU): the CPU path one GPU of this line "
                    f"replaces; {world_n} GPU(s) replace up to {world_n}x this" if world_n > 1 else
                    "the host CPU share of the one GPU (16 CPUs per GPU)")
        except Exception as e:  # a missing/failed baseline must not hide the GPU number
            log("cpu_baseline failed:", e)
            line["cpu_baseline"] = None
    parallel.barrier(world)                       # the other ranks wait for rank 0's CPU legs
    if rank == 0:
        emit_line(line)
    parallel.shutdown(world)
    return 0


def dry_run(args, world, parallel):
    """CPU plumbing rehearsal (gloo): shard spans of configs[3], the MAX / gather reductions
    and the line shape; no library call, no device."""
    import torch
    span = parallel.shard(args.global_batch, world.rank, world.size)
    recs = parallel.gather_objects(world, {"rank": world.rank, "span": list(span), "pid": os.getpid()})
    wall = parallel.reduce_max(world, 0.001 * (1 + world.rank))
    line = None
    if world.rank == 0:
        spans = [r["span"] for r in sorted(recs, key=lambda r: r["rank"])]
        line = {"metric": METRIC, "n_gpus": world.size, "ranks": world.size, "dry_run": True,
                "dist_backend": world.backend, "spans": spans, "pids": [r["pid"] for r in recs],
                "max_wall_s": wall, "scaling": args.scaling, "global_batch": args.global_batch}
    if args.scatter:
        # the scatter leg's plumbing on a small host batch: row i holds words 8 i .. 8 i + 7
        G = min(args.global_batch, 4096)
        sp = [parallel.shard(G, r, world.size) for r in range(world.size)]
        full = torch.arange(G * 8, dtype=torch.int32).view(G, 8) if world.rank == 0 else None
        out = torch.empty((sp[world.rank][1], 8), dtype=torch.int32)
        parallel.scatter_rows(world, full, sp, out)
        s0, c0 = sp[world.rank]
        ok = bool(torch.equal(out, torch.arange(s0 * 8, (s0 + c0) * 8, dtype=torch.int32).view(c0, 8)))
        oks = parallel.gather_objects(world, ok)
        if line is not None:
            line["scatter"] = {"rows": G, "slices_verified": bool(all(oks)), "ranks": world.size}
    if world.rank == 0 and not args.no_cpu_baseline:
        secs = args.cpu_secs or 0.2
        line["cpu_baseline"] = cpu_baseline("cfft_f32_1024", 1024, secs, secs)
    parallel.barrier(world, sync_device=False)
    if line is not None:
        emit_line(line)
    parallel.shutdown(world)
    return 0


def pmc_field(name, field, launch_items=None):
    """A field of the committed rocprofv3 PMC record `name` (profiles/pmc_traffic.json,
    written by tools/profile_collect.py), or None.  launch_items: the items (transforms,
    filters, matrices) one launch of this run processes; the record is used only when its
    profiled run launched the same number."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    rec = json.load(open(p)).get(name, {})
    cfg = rec.get("bench_config") or {}
    items = cfg.get("batch_per_gpu", cfg.get("global_batch"))
    if launch_items is not None and items != launch_items:
        return None
    return rec.get(field)


def valu_issue(name, launch_items, kern_ms):
    """Compute roofline of a VALU-issue-bound kernel from the committed PMC record `name`:
    SQ_INSTS_VALU per launch x the kernel's issue cycles per VALU instruction (full rate 2, half
    rate 4, transcendental 8 cycles per wave64 instruction, classes from its hottest loop's ISA,
    tools/profile_collect.py) against 256 CU x 4 SIMD x 2.4 GHz issue cycles per second, over
    this run's live kernel time."""
    cyc = pmc_field(name, "valu_issue_cycles_per_launch", launch_items)
    if cyc is None or not kern_ms:
        return None
    peak = 256 * 4 * 2.4e9
    ach = cyc / (kern_ms * 1e-3)
    return {"valu_insts_per_launch": pmc_field(name, "valu_insts_per_launch", launch_items),
            "issue_cycles_per_launch": round(cyc), "achieved": round(ach * 1e-12, 4), "peak": round(peak * 1e-12, 4),
            "unit": "T SIMD issue cycles/s (256 CU x 4 SIMD x 2.4 GHz)", "frac": round(ach / peak, 4),
            "source": pmc_field(name, "source", launch_items)}


def pmc_traffic(name, launch_items=None):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, when present."""
    return pmc_field(name, "hbm_bytes_per_launch", launch_items)


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    if args.gpus and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, argv)
    reserve_stdout()
    return main_rank(args)


if __name__ == "__main__":
    sys.exit(main())
