"""GPU: bench.py under a real RCCL process group.  RCCL cannot hold two ranks on
one device, so on a one-GPU box the `nccl` backend is exercised with a one-rank group
(CMSISDSP_DIST_SINGLE=1): process-group init on the device, the barrier + MAX all-reduce
around the timed region, the digest all-gather behind the checksum of checksums and the
configs[3] scatter leg all run through RCCL on device tensors, and the line must still be
bit-exact.  The 2..8-rank runs are the driver's; tests/test_bench_launcher.py covers the
N-rank plumbing with gloo."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_bench_one_rank_rccl_group(torch_gpu):
    env = dict(os.environ)
    env.update({"CMSISDSP_DIST_SINGLE": "1", "RANK": "0", "LOCAL_RANK": "0", "WORLD_SIZE": "1",
                "LOCAL_WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(_free_port())})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2", "--warmup", "1",
                        "--batch", "65536", "--global-batch", "65536", "--scatter", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout[-2000:]   # RCCL's banner goes to stderr
    line = json.loads(lines[0])
    assert line["dist_backend"] == "nccl" and line["n_gpus"] == 1 and line["devices_used"] == 1
    assert line["parity"]["bit_exact"] and line["parity"]["ranks_checked"] == 1
    for kind in ("q31", "q15"):
        c3 = line["config3"][kind]
        assert c3["parity"]["bit_exact"]
        assert c3["scatter"]["slices_verified"] and c3["scatter"]["ranks"] == 1
