"""Probe: does splitting one headline step (arm_cfft_f32 N=1024, 2^20 transforms in place) into
P concurrent launches on P streams move more bytes per second than one launch?  (The 2-rank
rehearsal on one GPU moved 6.47 TB/s aggregate against 6.11 single-process.)  Prints TB/s per
mode, alternated over rounds.  Results are not checked here (same kernel, same data layout)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "cmsis-dsp_amd"))
import cmsisdsp_amd as dsp  # noqa: E402

S = dsp.const_instance("arm_cfft_sR_f32_len1024")
B = 1 << 20
x = (torch.rand(B * 2048, device="cuda") - 0.5).view(B, 2048)
streams = [torch.cuda.Stream() for _ in range(8)]
cur = torch.cuda.current_stream()


def step(parts, flag):
    if parts == 1:
        dsp.cfft_batch(S, x, flag, 1)
        return
    ev = torch.cuda.Event()
    ev.record(cur)
    for i, c in enumerate(x.chunk(parts)):
        st = streams[i]
        st.wait_event(ev)
        dsp.cfft_batch(S, c, flag, 1, stream=st)
    for i in range(parts):
        cur.wait_stream(streams[i])


def serial(parts, flag):
    for c in x.chunk(parts):
        dsp.cfft_batch(S, c, flag, 1)


for k in range(30):
    step(1, k & 1)
torch.cuda.synchronize()
modes = [("1 launch", lambda f: step(1, f)), ("2 streams", lambda f: step(2, f)), ("4 streams", lambda f: step(4, f)),
         ("2 serial", lambda f: serial(2, f)), ("8 streams", lambda f: step(8, f))]
res = {m: [] for m, _ in modes}
for rnd in range(3):
    for name, fn in modes:
        for k in range(4):
            fn(k & 1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        steps = 20
        for k in range(steps):
            fn(k & 1)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[name].append(steps * 16.0 * B * 1024 / dt * 1e-12)
for name, v in res.items():
    print(f"{name:10s} " + " ".join(f"{t:.3f}" for t in v) + " TB/s")
