"""World-size-2 gloo test of the multi-GPU path's host logic (lazydb_amd.multi): one file per
rank, max-over-ranks timing, summed bytes, and the single tuple gather to rank 0. The per-rank
scan is the CPU oracle here (this container has no GPU); the GPU run uses the same module with
backend "nccl" (RCCL) in bench.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lazydb_amd import multi
        from oracle import coracle
        fids = multi.files_for_rank(list(range(1, 2 * world + 1)), rank, world)
        bufs, nbytes, nent = [], 0, 0
        for fid in fids:
            img, n, end = coracle.gen_log(1 << 18, 100 + fid, ksize=16, vsize=48)
            res, tup = coracle.scan(img, 0, fid=fid)
            bufs.append(np.frombuffer(tup.tobytes(), np.uint8))
            nbytes += int(res.end_off)
            nent += int(res.n_entries)
        mine = torch.from_numpy(np.concatenate(bufs).copy())
        t = multi.max_over_ranks(0.5 + rank, "cpu")
        tot = multi.sum_over_ranks([nbytes, nent], "cpu")
        got = multi.gather_tuples(mine)
        if rank == 0:
            q.put((t, tot, [g.numpy().tobytes() for g in got]))
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_matches_per_file_scans():
    from lazydb_amd import multi
    from oracle import coracle
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, tot, got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == pytest.approx(1.5)
    exp_bytes = exp_ent = 0
    for r in range(world):
        exp = b""
        for fid in multi.files_for_rank(list(range(1, 2 * world + 1)), r, world):
            img, n, end = coracle.gen_log(1 << 18, 100 + fid, ksize=16, vsize=48)
            res, tup = coracle.scan(img, 0, fid=fid)
            exp += tup.tobytes()
            exp_bytes += int(res.end_off)
            exp_ent += int(res.n_entries)
        assert got[r] == exp
    assert tot == [float(exp_bytes), float(exp_ent)]


def test_files_for_rank_round_robin():
    from lazydb_amd import multi
    assert multi.files_for_rank([5, 1, 3, 2, 4], 0, 2) == [1, 3, 5]
    assert multi.files_for_rank([5, 1, 3, 2, 4], 1, 2) == [2, 4]
    assert multi.files_for_rank([1], 1, 8) == []


def _gatherv_worker(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lazydb_amd import multi
        # unequal byte counts, one rank with nothing: the gatherv ships exactly the bytes (no padding)
        sizes = [48, 0, 16 * 1001]
        mine = torch.arange(sizes[rank], dtype=torch.int64).to(torch.uint8) ^ rank
        got = multi.gather_tuples(mine)
        if rank == 0:
            q.put(([g.numpy().tobytes() for g in got], multi.gather_tuples.last_bytes))
    finally:
        dist.destroy_process_group()


def test_three_rank_gatherv_unequal_sizes():
    world = 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gatherv_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, moved = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sizes = [48, 0, 16 * 1001]
    for r, g in enumerate(got):
        assert g == (torch.arange(sizes[r], dtype=torch.int64).to(torch.uint8) ^ r).numpy().tobytes()
    assert moved == sizes[1] + sizes[2]   # exactly the other ranks' bytes crossed to rank 0


def _gather_bad_worker(rank, world, port, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from lazydb_amd import multi
        # rank 1 hands in int32 tuples instead of bytes: every rank raises, none waits in the gather
        mine = torch.zeros(64, dtype=torch.uint8 if rank != 1 else torch.int32)
        try:
            multi.gather_tuples(mine)
            q.put((rank, "ok"))
        except RuntimeError as e:
            q.put((rank, "refused: " + str(e)))
    finally:
        dist.destroy_process_group()


def test_gatherv_refuses_on_every_rank():
    """the gather fails loudly on every rank, not with one rank raising and the others
    hanging in the collective."""
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gather_bad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(v.startswith("refused") for v in got.values()), got
