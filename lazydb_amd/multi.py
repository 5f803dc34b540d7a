"""Multi-GPU plumbing for the scan.

Log files are independent (every replay chain starts at offset 0, index.go:68-95), so ranks
scan disjoint files with no collective on the scan path (weak scaling). The only data exchange
is the single gather of index tuples to rank 0 — RCCL over xGMI on GPUs (backend "nccl"),
gloo in the CPU tests — plus scalar reductions of the timing.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def files_for_rank(fids, rank: int, world: int):
    """Round-robin files by fid; each rank keeps ascending fid order (index.go:103-108 order)."""
    return sorted(fids)[rank::world]


def coll_device(device):
    """Where collective buffers live: the GPU under RCCL; host memory under gloo (CPU tests, and
    the bench's one-GPU rehearsal of the N>1 path)."""
    if dist.is_initialized() and dist.get_backend() == "gloo":
        return torch.device("cpu")
    return device


def max_over_ranks(x: float, device) -> float:
    device = coll_device(device)
    t = torch.tensor([x], dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(xs, device):
    device = coll_device(device)
    t = torch.tensor(list(xs), dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


def gather_tuples(tuple_bytes: torch.Tensor, dst: int = 0):
    """Gather every rank's tuple byte buffer (uint8, 1-D, on the rank's device) to `dst`: a gatherv.

    One all_gather of the byte counts, then point-to-point transfers of exactly those bytes (one
    batched group of isend / irecv: over RCCL the receives run concurrently on dst's xGMI links), so
    unequal files ship no padding. Returns the list of per-rank buffers (rank order) on `dst`, None
    elsewhere; gather_tuples.last_bytes is the byte total that crossed to dst.
    """
    assert tuple_bytes.dtype == torch.uint8 and tuple_bytes.dim() == 1
    world = dist.get_world_size()
    rank = dist.get_rank()
    tuple_bytes = tuple_bytes.to(coll_device(tuple_bytes.device)).contiguous()
    dev = tuple_bytes.device
    n = torch.tensor([tuple_bytes.numel()], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    gather_tuples.last_bytes = sum(c for r, c in enumerate(counts) if r != dst)
    if rank == dst:
        bufs = [tuple_bytes if r == dst else torch.empty(counts[r], dtype=torch.uint8, device=dev)
                for r in range(world)]
        ops = [dist.P2POp(dist.irecv, bufs[r], r) for r in range(world) if r != dst and counts[r]]
    else:
        bufs = None
        ops = [dist.P2POp(dist.isend, tuple_bytes, dst)] if counts[rank] else []
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return bufs


gather_tuples.last_bytes = 0
