"""Where an i8-plane GEMM workgroup spends its time (diagnostic).

Runs arm_mat_mult_q15 / _q31 (1024^3 x 64, the bench shape) through a library built with
-DMI355X_I8_STAMPS=1 (tools/build_variant.sh stamps "-DMI355X_I8_STAMPS=1"), whose
mat_mult_i8v2_kernel records s_memtime per workgroup after the tile decode, the prologue, the K
loop, the epilogue arithmetic and the copy-out, and prints per-phase medians (cycles and us at the
clock measured by s_memtime / s_memrealtime) and the gap between consecutive workgroups on a CU.
Usage: python tools/probes/i8_phases.py cmsis-dsp_amd/lib/variants/lib_stamps.so
"""
import ctypes
import json
import os
import sys

import numpy as np

LIB = os.path.abspath(sys.argv[1])
os.environ["CMSISDSP_MI355X_LIB"] = LIB
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "cmsis-dsp_amd"))
import torch  # noqa: E402
import cmsisdsp_amd as dsp  # noqa: E402

lib = ctypes.CDLL(LIB)
lib.arm_mi355x_i8_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
out = {}
for kind, dt, bits, tiles in (("q15", torch.int16, 15, 64 * 64), ("q31", torch.int32, 31, 64 * 128)):
    g = torch.Generator(device="cuda").manual_seed(3)
    A = torch.randint(-(1 << bits), (1 << bits) - 1, (64, 1024, 1024), dtype=dt, device="cuda", generator=g)
    B = torch.randint(-(1 << bits), (1 << bits) - 1, (64, 1024, 1024), dtype=dt, device="cuda", generator=g)
    C = torch.empty_like(A)
    for _ in range(3):
        dsp.mat_mult_batch(A, B, C)
    torch.cuda.synchronize()
    st = np.zeros((tiles, 8), np.uint64)
    assert lib.arm_mi355x_i8_stamps(st.ctypes.data, tiles) == 0
    t = st[:, :5].astype(np.int64)
    clock = np.median((t[:, 4] - t[:, 0]) / ((st[:, 6].astype(np.int64) - st[:, 5].astype(np.int64)) / 100e6))
    ph = {"prologue": t[:, 1] - t[:, 0], "k_loop": t[:, 2] - t[:, 1], "epilogue_math": t[:, 3] - t[:, 2],
          "copy_out": t[:, 4] - t[:, 3], "workgroup": t[:, 4] - t[:, 0]}
    rec = {"clock_ghz": float(clock / 1e9)}
    for k, v in ph.items():
        rec[k + "_cycles_median"] = float(np.median(v))
        rec[k + "_us_median"] = float(np.median(v) / clock * 1e6)
    # gaps between consecutive workgroups on one CU (hw_id CU/SE bits + XCC id)
    hw = st[:, 7]
    cu = ((hw & 0xFFFFFFFF) >> 8) & 0xFF | ((hw >> 32) & 0xF) << 8
    gaps, spans, busy = [], [], []
    for c in np.unique(cu):
        idx = np.where(cu == c)[0]
        s0 = t[idx, 0]
        order = np.argsort(s0)
        starts, ends = t[idx, 0][order], t[idx, 4][order]
        if len(idx) > 1:
            gaps.extend((starts[1:] - ends[:-1]).tolist())
        spans.append(ends.max() - starts.min())
        busy.append((ends - starts).sum())
    rec["cus_seen"] = int(len(np.unique(cu)))
    rec["gap_cycles_median"] = float(np.median(gaps)) if gaps else None
    rec["cu_busy_fraction_median"] = float(np.median(np.array(busy) / np.array(spans)))
    rec["k_steps"] = 1024 // 64
    rec["k_step_cycles_median"] = rec["k_loop_cycles_median"] / rec["k_steps"]
    out[kind] = rec
print(json.dumps(out))
