"""CPU: bench.py's N-rank launch (SURVEY §8e / the bench contract).  `bench.py --gpus 2`
without a torchrun environment must start two ranks as child processes (torch.distributed.run),
shard the configs[3] global batch in contiguous slices and print one line with n_gpus 2; a
world size that disagrees with --gpus must fail loudly instead of measuring fewer GPUs."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus2_launches_two_ranks_strong_spans():
    r = _run(["--gpus", "2", "--dry-run", "--scaling", "strong", "--global-batch", "1048576"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["ranks"] == 2 and line["dist_backend"] == "gloo"
    assert len(set(line["pids"])) == 2 and os.getpid() not in line["pids"]
    assert line["spans"] == [[0, 524288], [524288, 524288]]
    assert line["max_wall_s"] == 0.002          # MAX over ranks (rank r reports 0.001 * (r + 1))


def test_gpus2_scatter_leg_and_cpu_baseline():
    """N > 1 lines carry rank 0's cpu_baseline, and --scatter moves each rank its contiguous
    slice of the global batch from rank 0 (point-to-point; gloo on CPU here)."""
    r = _run(["--gpus", "2", "--dry-run", "--scaling", "strong", "--global-batch", "1000", "--scatter",
              "--cpu-secs", "0.2"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["scatter"] == {"rows": 1000, "slices_verified": True, "ranks": 2}
    cb = line["cpu_baseline"]
    if os.path.exists(os.path.join(ROOT, "oracle", "_ref", "bench_ref")):
        assert cb["kind"] == "reference" and cb["value"] > 0 and cb["cores"] >= 1 and cb["affinity_cpus"] >= 1


def test_gpus3_ragged_global_batch():
    r = _run(["--gpus", "3", "--dry-run", "--scaling", "strong", "--global-batch", "10"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = _line(r.stdout)
    assert line["n_gpus"] == 3
    assert line["spans"] == [[0, 4], [4, 3], [7, 3]]


def test_world_size_mismatch_fails_loudly():
    r = _run(["--gpus", "2", "--dry-run"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)


def test_driver_style_torchrun_stdout_is_one_json_line():
    """The driver runs `python -m torch.distributed.run ... bench.py --gpus N` itself (no
    launcher in between): whatever the ranks' libraries print (gloo / RCCL banners) must reach
    stderr, and stdout must hold exactly rank 0's JSON line."""
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--dry-run", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks"] == 2
