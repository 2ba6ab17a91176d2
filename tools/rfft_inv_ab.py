#!/usr/bin/env python3
"""Timing of the batched inverse arm_rfft_q31 / _q15 (spectrum rows [batch][2N] -> [batch][N]) for
A/B runs of library builds (CMSISDSP_MI355X_LIB).  2^29 output samples per launch at every N,
full-range random spectra, 20 warmup + 20 timed launches on HIP events; one line per (kind, N):
kind N Gsamples/s avg_ms.  Parity is the GPU tests' job (tests/test_rfft_fixed.py)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cmsis-dsp_amd"))
import torch  # noqa: E402
import cmsisdsp_amd as dsp  # noqa: E402

ns = [int(a) for a in sys.argv[1:]] or [512, 1024, 2048, 4096, 8192]
for kind, dt in (("q31", torch.int32), ("q15", torch.int16)):
    for n in ns:
        S = dsp.arm_rfft_instance_q31() if kind == "q31" else dsp.arm_rfft_instance_q15()
        assert getattr(dsp, f"arm_rfft_init_{kind}")(S, n, 1, 1) == 0
        batch = (1 << 29) // n
        info = torch.iinfo(dt)
        src = torch.randint(info.min, info.max, (batch, 2 * n), dtype=dt, device="cuda")
        dst = torch.empty((batch, n), dtype=dt, device="cuda")
        for _ in range(20):
            dsp.rfft_fixed_batch(S, src, dst)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            dsp.rfft_fixed_batch(S, src, dst)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"{kind} {n} {batch * n / ms / 1e6:.1f} {ms:.4f}", flush=True)
        del src, dst
