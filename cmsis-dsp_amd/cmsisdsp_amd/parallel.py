"""Multi-GPU plumbing for batched DSP: one process per GPU, no data-path collective.

The reference library is single-threaded and has no parallelism; the only
axis that scales is the batch of independent transforms / filters / matrices (§8e).
Every rank owns a contiguous slice of the global batch and generates (or receives) its
own data, so the hot path never communicates.  Collectives are used only around it:
  * a barrier + MAX reduction of the timed interval (bench contract),
  * an all-gather of per-rank parity digests ("checksum of checksums") so rank 0 can
    assert that every shard matched the reference bit for bit,
  * the separately timed scatter leg of SURVEY §8e (scatter_rows: rank 0 holds a global
    batch and sends each rank its contiguous slice point to point, RCCL over xGMI), which
    is reported beside the compute, never inside it.
Backends: "nccl" (= RCCL over xGMI on ROCm) on GPUs, "gloo" for CPU rehearsals and tests.
Nothing here touches the HIP kernels; tests/test_dist.py runs it with gloo, world size 2.
"""
import os
from dataclasses import dataclass

import numpy as np


@dataclass
class World:
    rank: int = 0
    size: int = 1
    local_rank: int = 0
    backend: str = "none"

    @property
    def distributed(self):
        return self.backend != "none"


def init(backend=None, device=True):
    """Initialise from the torchrun environment (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_*).
    device=True pins the process to GPU local_rank % device_count (the HIP device the
    library's launches then use)."""
    import torch
    import torch.distributed as dist
    size = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_size = int(os.environ.get("LOCAL_WORLD_SIZE", str(size)))
    ndev = torch.cuda.device_count() if device else 0
    if device:
        torch.cuda.set_device(local % max(1, ndev))
    # CMSISDSP_DIST_SINGLE=1: build the process group even for one rank, so the RCCL path
    # (init, barrier, MAX all-reduce, digest all-gather, scatter) runs on a one-GPU box, where
    # RCCL cannot hold two ranks on one device (tests/test_gpu_dist_nccl.py).
    if size == 1 and os.environ.get("CMSISDSP_DIST_SINGLE") != "1":
        return World(rank, size, local, "none")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        # RCCL needs one GPU per rank; more local ranks than GPUs is a rehearsal -> gloo
        backend = "nccl" if device and ndev >= local_size else "gloo"
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
    else:
        dist.init_process_group("gloo")
    return World(rank, size, local, backend)


def shutdown(world):
    if world.distributed:
        import torch.distributed as dist
        dist.destroy_process_group()


def shard(total, rank, size):
    """Contiguous slice [start, start+count) of `total` items for `rank` (balanced: the
    first total % size ranks get one extra)."""
    base, extra = divmod(total, size)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def weak_offset(per_rank, rank):
    """Global index of a rank's first item when every rank processes `per_rank` items."""
    return per_rank * rank


def seed_for(rank, salt=0):
    """Per-rank generator seed: 0x5EED + a large prime stride (disjoint streams)."""
    return 0x5EED + 1000003 * rank + salt


def block_seed(block, salt=0):
    """Seed of global block `block` of a batch whose content must not depend on the world
    size (strong scaling): every rank regenerates the blocks its slice overlaps."""
    return 0x5EED0000 + 7919 * block + 1000003 * salt


def _tensor_for(world, value, dtype):
    import torch
    dev = "cuda" if world.backend == "nccl" else "cpu"
    return torch.tensor([value], dtype=dtype, device=dev)


def barrier(world, sync_device=True):
    import torch
    if sync_device and torch.cuda.is_available():
        torch.cuda.synchronize()
    if world.distributed:
        import torch.distributed as dist
        dist.barrier()
    if sync_device and torch.cuda.is_available():
        torch.cuda.synchronize()


def reduce_max(world, x):
    if not world.distributed:
        return float(x)
    import torch
    import torch.distributed as dist
    t = _tensor_for(world, float(x), torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(world, x):
    if not world.distributed:
        return float(x)
    import torch
    import torch.distributed as dist
    t = _tensor_for(world, float(x), torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def digest(arr):
    """64-bit digest of an array's bytes (xxh64, order-sensitive within the array)."""
    import xxhash
    return xxhash.xxh64(np.ascontiguousarray(arr).tobytes()).intdigest()


def gather_objects(world, obj):
    """All-gather of a small Python object (per-rank parity record)."""
    if not world.distributed:
        return [obj]
    import torch.distributed as dist
    out = [None] * world.size
    dist.all_gather_object(out, obj)
    return out


def scatter_rows(world, full, spans, out):
    """Rank 0 holds `full` (the global batch, rows = items) and every rank r receives rows
    [spans[r][0], spans[r][0] + spans[r][1]) into `out`; rank 0 copies its own slice.  The
    sends are posted together (batch_isend_irecv: with nccl one RCCL group of point-to-point
    transfers over xGMI, rank 0 -> each peer on its own link); gloo moves CPU tensors."""
    s0, c0 = spans[world.rank]
    if not world.distributed:
        out.copy_(full[s0:s0 + c0])
        return
    import torch.distributed as dist
    ops = []
    if world.rank == 0:
        for r in range(1, world.size):
            s, c = spans[r]
            if c:
                ops.append(dist.P2POp(dist.isend, full[s:s + c], r))
    elif c0:
        ops.append(dist.P2POp(dist.irecv, out, 0))
    reqs = dist.batch_isend_irecv(ops) if ops else []
    if world.rank == 0 and c0:
        out.copy_(full[s0:s0 + c0])
    for q in reqs:
        q.wait()


def checksum_of_checksums(records):
    """Combine per-rank (rank, gpu_digest, ref_digest) records: returns (all_equal,
    combined digest over ranks in rank order)."""
    import xxhash
    recs = sorted(records, key=lambda r: r["rank"])
    h = xxhash.xxh64()
    for r in recs:
        h.update(int(r["gpu_digest"]).to_bytes(8, "little"))
    return all(r["gpu_digest"] == r["ref_digest"] for r in recs), h.intdigest()
