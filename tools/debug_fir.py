"""Debug helper: FIR batched vs the reference build, prints the mismatching output ranges."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cmsis-dsp_amd"), os.path.join(ROOT, "tests")]
import torch
import refs
import cmsisdsp_amd as dsp
from test_gpu_rfft_fir_mat import _fir_batched

ref = refs.ref_lib()
kind = sys.argv[1] if len(sys.argv) > 1 else "f32"
for taps, block in [(1024, 3000), (1023, 3000), (1000, 3000), (1024, 2048), (512, 3000), (1024, 5000)]:
    rng = np.random.default_rng(taps * 7 + block)
    coeffs = (rng.standard_normal(taps) / np.sqrt(taps)).astype(np.float32)
    blocks = [[rng.uniform(-1, 1, block).astype(np.float32) for _ in range(2)] for _ in range(3)]
    got, hist = _fir_batched(dsp, torch, kind, coeffs, blocks)
    for f in range(3):
        want, state = ref.fir(kind, coeffs, blocks[f])
        for k in range(2):
            bad = np.nonzero(got[k][f].view(np.uint32) != want[k].view(np.uint32))[0]
            if len(bad):
                print(taps, block, "filter", f, "call", k, "bad", len(bad), "first", bad[:5], "last", bad[-3:],
                      "got", got[k][f][bad[:3]], "want", want[k][bad[:3]])
        if hist[f].tobytes() != state[:taps - 1].tobytes():
            print(taps, block, "filter", f, "history differs")
print("done")
