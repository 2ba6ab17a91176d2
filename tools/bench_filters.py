#!/usr/bin/env python3
"""Throughput of the filtering functions outside bench.py's workloads (round 2 additions):
arm_fir_q7, arm_fir_decimate_*, arm_fir_interpolate_*, arm_fir_sparse_*, arm_fir_lattice_* through the batched device API on one
GPU, HIP-event timed on the launch stream after a clock-settle phase, each with a bit-exact
check of 2 streams against the CPU checker (the reference build when present).
Usage: python tools/bench_filters.py [name ...]  -> one JSON line per workload."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cmsis-dsp_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import cmsisdsp_amd as dsp  # noqa: E402
from cmsisdsp_amd import _abi  # noqa: E402
import refs  # noqa: E402

BATCH, BLOCK, TAPS = 1 << 16, 4096, 128
SP_TAPS, SP_DELAY = 32, 1024            # sparse: 32 nonzero taps at delays in [0, 1024]
LAT_STAGES = 32                         # lattice: 32 stages
# name: (function, factor, dtype)
CASES = {
    "fir_q7": ("q7", 1, "q7"),
    "fir_decimate_f32_m4": ("decimate_f32", 4, "f32"),
    "fir_decimate_q15_m4": ("decimate_q15", 4, "q15"),
    "fir_decimate_fast_q31_m4": ("decimate_fast_q31", 4, "q31"),
    "fir_decimate_q31_m4": ("decimate_q31", 4, "q31"),
    "fir_interpolate_f32_l4": ("interpolate_f32", 4, "f32"),
    "fir_interpolate_q31_l4": ("interpolate_q31", 4, "q31"),
    "fir_sparse_f32": ("sparse_f32", 1, "f32"),
    "fir_sparse_q31": ("sparse_q31", 1, "q31"),
    "fir_sparse_q15": ("sparse_q15", 1, "q15"),
    "fir_sparse_q7": ("sparse_q7", 1, "q7"),
    "fir_lattice_f32": ("lattice_f32", 1, "f32"),
    "fir_lattice_q31": ("lattice_q31", 1, "q31"),
    "fir_lattice_q15": ("lattice_q15", 1, "q15"),
}
TDT = {"f32": torch.float32, "q15": torch.int16, "q31": torch.int32, "q7": torch.int8}


def checker():
    try:
        return refs.ref_lib(), "reference"
    except (FileNotFoundError, OSError):
        return refs.oracle_lib(), "oracle"


def timed(launch, steps=10, warmup=3, settle_ms=40.0):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(64):
        launch()
        e1.record(st)
        e1.synchronize()
        if e0.elapsed_time(e1) >= settle_ms:
            break
    for _ in range(warmup):
        launch()
    e0.record(st)
    for _ in range(steps):
        launch()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / steps


def run(name):
    fn, factor, kind = CASES[name]
    rng = np.random.default_rng(7)
    dt = refs.DTYPE[kind]
    sparse = fn.startswith("sparse")
    lattice = fn.startswith("lattice")
    taps = SP_TAPS if sparse else LAT_STAGES if lattice else TAPS
    if lattice and kind == "f32":
        c = rng.uniform(-0.9, 0.9, taps).astype(np.float32)
    elif kind == "f32":
        c = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
    else:
        info = np.iinfo(dt)
        c = rng.integers(info.min, info.max, taps, endpoint=True).astype(dt)
    delays = np.sort(rng.choice(SP_DELAY + 1, taps, replace=False)).astype(np.int32)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    if kind == "f32":
        src = torch.rand((BATCH, BLOCK), generator=g, device="cuda") - 0.5
    else:
        info = np.iinfo(dt)
        src = torch.randint(int(info.min), int(info.max) + 1, (BATCH, BLOCK), generator=g, device="cuda",
                            dtype=torch.int64).to(TDT[kind])
    dc = torch.from_numpy(c.copy()).cuda()
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    if lattice:
        S = _abi.arm_fir_lattice_instance(numStages=taps, pState=None, pCoeffs=dc.data_ptr())
        H, nout, f = taps, BLOCK, getattr(dsp.lib, f"arm_fir_{fn}_batch")
    elif sparse:
        dd = torch.from_numpy(delays.copy()).cuda()
        S = _abi.arm_fir_sparse_instance(numTaps=taps, pCoeffs=dc.data_ptr(), maxDelay=SP_DELAY,
                                         pTapDelay=dd.data_ptr())
        H, nout, f = SP_DELAY, BLOCK, getattr(dsp.lib, f"arm_fir_{fn}_batch")
    elif fn == "q7":
        S = _abi.arm_fir_instance_q7(numTaps=TAPS, pState=None, pCoeffs=dc.data_ptr())
        H, nout, f = TAPS - 1, BLOCK, dsp.lib.arm_fir_q7_batch
    elif fn.startswith("decimate"):
        S = _abi.arm_fir_decimate_instance(M=factor, numTaps=TAPS, pCoeffs=dc.data_ptr(), pState=None)
        H, nout, f = TAPS - 1, BLOCK // factor, getattr(dsp.lib, f"arm_fir_{fn}_batch")
    else:
        S = _abi.arm_fir_interpolate_instance(L=factor, phaseLength=TAPS // factor, pCoeffs=dc.data_ptr(),
                                              pState=None)
        H, nout, f = TAPS // factor - 1, BLOCK * factor, getattr(dsp.lib, f"arm_fir_{fn}_batch")
    dst = torch.empty((BATCH, nout), dtype=TDT[kind], device="cuda")
    hist = torch.zeros((BATCH, H), dtype=TDT[kind], device="cuda")

    def launch(d=dst, h=hist, s=src, b=BATCH):
        rc = f(C.byref(S), C.c_void_p(s.data_ptr()), C.c_void_p(d.data_ptr()), BLOCK, b, C.c_void_p(h.data_ptr()),
               stream)
        assert rc == 0, dsp.last_error()

    ms = timed(launch)
    host, hk = checker()
    d2 = torch.empty((2, nout), dtype=TDT[kind], device="cuda")
    h2 = torch.zeros((2, H), dtype=TDT[kind], device="cuda")
    launch(d2, h2, src[:2].contiguous(), 2)
    torch.cuda.synchronize()
    ok = True
    for i in range(2):
        x = src[i].cpu().numpy()
        if lattice:
            want = host.lattice(kind, c, [x])[0][0]
        elif sparse:
            want = host.sparse(kind, c, delays, SP_DELAY, [x])[0][0]
        elif fn == "q7":
            want = host.fir("q7", c, [x])[0][0]
        else:
            want = host.multirate(fn, factor, c, [x])[1][0]
        ok &= d2[i].cpu().numpy().tobytes() == want.tobytes()
    macs = BATCH * (BLOCK * taps * (2 if lattice else 1) if fn == "q7" or sparse or lattice else (BLOCK // factor) * TAPS if fn.startswith("decimate")
                    else BLOCK * TAPS)
    esz = np.dtype(dt).itemsize
    extra = {"maxDelay": SP_DELAY} if sparse else {"numStages": taps} if lattice else {}
    return {"workload": name, "function": f"arm_fir_{fn}", "numTaps": taps, **extra, "factor": factor, "blockSize": BLOCK,
            "batch": BATCH, "avg_kernel_ms": round(ms, 4),
            "input_gsamples_per_s": round(BATCH * BLOCK / (ms * 1e-3) * 1e-9, 2),
            "output_gsamples_per_s": round(BATCH * nout / (ms * 1e-3) * 1e-9, 2),
            "gmacs_per_s": round(macs / (ms * 1e-3) * 1e-9, 1),
            "hbm_gbs": round(BATCH * (BLOCK + nout) * esz / (ms * 1e-3) * 1e-9, 1),
            "bit_exact": bool(ok), "checker": hk}


if __name__ == "__main__":
    for name in sys.argv[1:] or list(CASES):
        print(json.dumps(run(name)), flush=True)
        torch.cuda.empty_cache()
