"""Drop-in C programs: the reference's FFT-bin example call sequence and the batched API,
compiled against include/ and linked to libcmsisdsp_mi355x.so (compile on CPU; run on GPU)."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "oracle", "_build")
LIBDIR = os.path.join(ROOT, "cmsis-dsp_amd", "lib")


def _build(name, hip=False):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, name)
    cmd = ["gcc", "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "examples", name + ".c"),
           "-L" + LIBDIR, "-lcmsisdsp_mi355x", "-lm", "-o", exe, "-Wl,-rpath," + LIBDIR]
    if hip:
        cmd[1:1] = ["-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
        cmd += ["-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    subprocess.run(cmd, check=True, capture_output=True)
    return exe


def test_examples_compile_and_link():
    assert os.path.exists(_build("fft_bin_dropin"))
    assert os.path.exists(_build("batched_cfft", hip=True))


@pytest.mark.gpu
@pytest.mark.parametrize("sync", ["spin", "sync"])
def test_fft_bin_example_runs_on_gpu(torch_gpu, sync):
    """Both completion modes of the synchronous calls (CMSISDSP_MI355X_SYNC): the spin on the
    coherent word the transform's workgroup writes, and a plain stream synchronisation."""
    exe = _build("fft_bin_dropin")
    x = np.load(os.path.join(ROOT, "tests", "golden", "reference_patterns.npz"))["kat_fftbin_input"]
    inp = os.path.join(OUT, "fftbin_input.f32")
    x.astype(np.float32).tofile(inp)
    env = dict(os.environ, CMSISDSP_MI355X_SYNC=sync)
    r = subprocess.run([exe, inp], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0 and r.stdout.strip() == "SUCCESS 213", r.stdout + r.stderr


@pytest.mark.gpu
def test_batched_example_runs_on_gpu(torch_gpu):
    exe = _build("batched_cfft", hip=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("OK"), r.stdout + r.stderr
