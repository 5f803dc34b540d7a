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


def gather_floats(xs, device):
    """Every rank's list of floats (same length on every rank), rank order, on every rank."""
    device = coll_device(device)
    t = torch.tensor([float(x) for x in xs], dtype=torch.float64, device=device)
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return [[float(v) for v in t.tolist()]]
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[float(v) for v in o.tolist()] for o in out]


def agree(ok: bool, what: str, device) -> None:
    """Every rank learns whether every rank's local check passed (one all_reduce MIN of a flag) and all
    of them raise together: a rank that raised alone before a collective would leave the others blocked
    in it (under RCCL until the process-group timeout), so checks on a rank's own inputs go through here
    before the collective they guard."""
    t = torch.tensor([1 if ok else 0], dtype=torch.int64, device=coll_device(device))
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    if int(t.item()) == 0:
        raise RuntimeError(f"{what}: refused on every rank (a rank's own check failed"
                           f"{'' if not ok else ', not this one'})")


def gather_tuples(tuple_bytes: torch.Tensor, dst: int = 0, device=None):
    """Gather every rank's tuple byte buffer (uint8, 1-D, on the rank's device) to `dst`: a gatherv.

    One all_gather of the byte counts, then point-to-point transfers of exactly those bytes (one
    batched group of isend / irecv: over RCCL the receives run concurrently on dst's xGMI links), so
    unequal files ship no padding. Returns the list of per-rank buffers (rank order) on `dst`, None
    elsewhere; gather_tuples.last_bytes is the byte total that crossed to dst. A rank whose buffer is
    not a 1-D uint8 tensor makes every rank raise (agree) instead of leaving the others blocked.
    `device`: the rank's GPU (default: the buffer's device), where the collective buffers live under RCCL.
    """
    world = dist.get_world_size()
    rank = dist.get_rank()
    ok = isinstance(tuple_bytes, torch.Tensor) and tuple_bytes.dtype == torch.uint8 and tuple_bytes.dim() == 1 \
        and 0 <= dst < world
    if device is None:
        device = tuple_bytes.device if isinstance(tuple_bytes, torch.Tensor) else \
            (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    dev = coll_device(device)
    agree(ok, "gather_tuples", dev)
    tuple_bytes = tuple_bytes.to(dev).contiguous()
    n = torch.tensor([tuple_bytes.numel()], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    # self-check: every rank sees its own count come back; a transport or caller fault makes
    # every rank raise instead of posting mismatched sends and receives
    agree(counts[rank] == tuple_bytes.numel(), "gather_tuples: byte counts", dev)
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
