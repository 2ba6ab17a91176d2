"""CPU, world size 2, gloo: the multi-GPU plumbing of bench.py (cmsisdsp_amd.parallel)
without GPU kernels.  Each rank transforms its contiguous shard of a global batch with the
oracle, digests it, and the all-gathered digests must equal what one process computes for
the whole batch ("checksum of checksums"); the timing reduction is a MAX over ranks."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from cmsisdsp_amd import parallel


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _global_batch(kind, n, total):
    import refs
    return np.stack([refs.rand_input(kind, 2 * n, seed=1000 + i) for i in range(total)])


def _worker(rank, size, port, kind, n, total, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(size), LOCAL_RANK=str(rank),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    try:
        import refs
        world = parallel.init(backend="gloo", device=False)
        start, count = parallel.shard(total, world.rank, world.size)
        x = _global_batch(kind, n, total)[start:start + count]
        y = refs.oracle_lib().cfft_many(kind, n, x, 0, 1)
        d = parallel.digest(y.view(np.uint8))
        recs = parallel.gather_objects(world, {"rank": rank, "gpu_digest": d, "ref_digest": d,
                                               "start": start, "count": count})
        tmax = parallel.reduce_max(world, 1.0 + rank)
        tsum = parallel.reduce_sum(world, count)
        parallel.barrier(world, sync_device=False)
        if rank == 0:
            q.put({"recs": recs, "tmax": tmax, "tsum": tsum})
        parallel.shutdown(world)
    except Exception as e:  # surface worker failures in the parent
        q.put({"error": repr(e)})
        raise


@pytest.mark.parametrize("kind,n,total", [("f32", 1024, 13), ("q31", 4096, 6)])
def test_sharded_batch_checksum_of_checksums(kind, n, total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, kind, n, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
    assert "error" not in res, res
    recs = sorted(res["recs"], key=lambda r: r["rank"])
    # shards are contiguous, disjoint and cover the batch
    assert recs[0]["start"] == 0 and recs[0]["start"] + recs[0]["count"] == recs[1]["start"]
    assert recs[1]["start"] + recs[1]["count"] == total and res["tsum"] == total
    assert res["tmax"] == 2.0
    # the per-rank digests combine to the single-process digests of the same shards
    import refs
    full = refs.oracle_lib().cfft_many(kind, n, _global_batch(kind, n, total), 0, 1)
    single = [{"rank": r["rank"], "gpu_digest": parallel.digest(full[r["start"]:r["start"] + r["count"]].view(np.uint8)),
               "ref_digest": 0} for r in recs]
    ok, combined = parallel.checksum_of_checksums(recs)
    _, combined_single = parallel.checksum_of_checksums(single)
    assert ok and combined == combined_single


def test_shard_arithmetic():
    for total in (0, 1, 7, 1 << 20):
        for size in (1, 2, 3, 8):
            spans = [parallel.shard(total, r, size) for r in range(size)]
            assert sum(c for _, c in spans) == total
            assert all(spans[i][0] + spans[i][1] == spans[i + 1][0] for i in range(size - 1))
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    assert len({parallel.seed_for(r) for r in range(8)}) == 8
    assert parallel.weak_offset(1 << 20, 3) == 3 << 20
