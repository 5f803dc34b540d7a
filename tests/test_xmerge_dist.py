"""Cross-GPU merge over real torch.distributed ranks (lazydb_amd.xmerge.merge_distributed).

* CPU (gloo, world 2 and 3): the variable-length all-gather that carries the summary logs and the
  entry sizes between ranks.
* GPU (gloo, world 2, both ranks on cuda:0 — the box has one GPU; the 8-GPU run uses RCCL with the
  same code): each rank merges its fid block; the pieces joined in rank order equal the oracle's
  single merge of every file, bit for bit."""
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


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _varlen_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from lazydb_amd.xmerge import _all_gather_varlen
        a = torch.arange(rank * 5, dtype=torch.uint8)                 # rank 0 sends nothing
        b = torch.full((rank + 1,), -rank - 7, dtype=torch.int32)
        ga = _all_gather_varlen(a, dist)
        gb = _all_gather_varlen(b, dist)
        q.put((rank, [x.tolist() for x in ga], [x.tolist() for x in gb]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_all_gather_varlen_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_varlen_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, ga, gb in got:
        assert ga == [list(range(r * 5)) for r in range(world)]
        assert gb == [[-r - 7] * (r + 1) for r in range(world)]


def _a2a_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        from lazydb_amd.xmerge import _all_to_all_varlen
        # rank r sends (r + 1) * o + 1 bytes of value 10 r + o to rank o (rank 0 sends nothing to rank 0)
        chunks = [torch.full(((rank + 1) * o + (0 if rank == 0 and o == 0 else 1),), 10 * rank + o, dtype=torch.uint8)
                  for o in range(world)]
        got = _all_to_all_varlen(chunks, dist, torch.device("cpu"))
        q.put((rank, [x.tolist() for x in got]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_all_to_all_varlen_gloo(world):
    """The hash-partitioned merge's exchange (xmerge._all_to_all_varlen) on the gloo path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_a2a_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, rows in got:
        for src, row in enumerate(rows):
            n = (src + 1) * rank + (0 if src == 0 and rank == 0 else 1)
            assert row == [10 * src + rank] * n


CASE = dict(seed=11, n_files=4, cap=32 << 20, n_records=4 * 101_000, max_file_size=8 << 20,
            p_delete=20_000, p_expire=50_000, ksize=64, vsize=256)


def _merge_worker(rank, world, port, q, hashed=False):
    _init(rank, world, port)
    try:
        from lazydb_amd import Engine
        from lazydb_amd import xmerge as X
        from tests import merge_cases as MC
        files, kw = MC.case_generated(**CASE)
        blk = np.array_split(np.arange(len(files)), world)[rank]
        eng = Engine(0)
        mine = [(torch.from_numpy(np.ascontiguousarray(files[i][0])).to("cuda:0"), files[i][1], files[i][2])
                for i in blk]
        if hashed:
            out = X.merge_hashed_distributed(eng, mine, kw["active_fid"], kw["active_off"], kw["max_file_size"],
                                             kw["now"])
        else:
            out = X.merge_distributed(eng, mine, max(f[1] for f in files), kw["active_fid"], kw["active_off"],
                                      kw["max_file_size"], kw["now"])
        q.put((rank, int(blk[0]), out["stream"].cpu().numpy().tobytes(), out["pos"].tobytes(),
               out["segments"].tobytes(), out["live"].cpu().numpy().tobytes(), out["start"], out["end"]))
        eng.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("hashed", [False, True])
def test_merge_distributed_two_ranks(hashed):
    """Summary exchange (hashed=False) and hash-partitioned liveness (hashed=True: route records and
    keys to the key owners, flags back, two all-to-alls) over two real ranks."""
    from oracle import coracle
    from tests import merge_cases as MC
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_merge_worker, args=(r, world, port, q, hashed)) for r in range(world)]
    for p in ps:
        p.start()
    got = sorted([q.get(timeout=240) for _ in range(world)])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    files, kw = MC.case_generated(**CASE)
    ref, stream, pos, segs, live, stats = coracle.merge(files, kw["active_fid"], kw["active_off"],
                                                        kw["max_file_size"], kw["now"])
    assert b"".join(g[2] for g in got) == stream.tobytes()
    gp = []
    for g in got:
        p = np.frombuffer(g[3], dtype=coracle.MERGE_POS).copy()
        p["src_file"] += g[1]
        gp.append(p)
    assert np.concatenate(gp).tobytes() == pos.tobytes()
    assert b"".join(g[5] for g in got) == live.tobytes()
    assert got[1][6] == got[0][7] and got[-1][7] == (ref.end_fid, ref.end_off)
    n_seg = sum(len(g[4]) // coracle.MERGE_SEGMENT.itemsize for g in got)
    assert n_seg in (ref.n_segments, ref.n_segments + 1)   # + 1 when the rank boundary splits a run


def _fid_block_worker(rank, world, port, q, blocks):
    _init(rank, world, port)
    try:
        from lazydb_amd.xmerge import check_fid_blocks
        files = [(None, f, False) for f in blocks[rank]]
        try:
            check_fid_blocks(files, dist)
            q.put((rank, "ok"))
        except ValueError as e:
            q.put((rank, "refused: " + str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("blocks,ok", [
    ([[0, 1], [2, 3]], True),
    ([[0, 1], []], True),                      # an empty block is skipped
    ([[0, 2], [1, 3]], False),                 # round-robin split: refused, not silently wrong
    ([[2, 3], [0, 1]], False),                 # blocks descending in rank order
    ([[1, 0], [2, 3]], False),                 # one rank's own fids descending: every rank raises (no hang)
    ([[0, 0], [2, 3]], False),                 # a duplicate fid on one rank
])
def test_fid_blocks_checked_gloo(blocks, ok):
    """Both cross-GPU merges take last-writer-wins order from rank order: a split whose
    fid blocks are not ascending by rank raises on every rank instead of producing wrong liveness."""
    world = len(blocks)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_fid_block_worker, args=(r, world, port, q, blocks)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        assert (got[r] == "ok") == ok, got


def _a2a_bad_worker(rank, world, port, q):
    _init(rank, world, port)
    try:
        import torch
        from lazydb_amd.xmerge import _all_to_all_varlen
        # rank 1 hands in one chunk too few: every rank must raise before any byte moves
        n = world if rank != 1 else world - 1
        chunks = [torch.full((3 + o,), rank, dtype=torch.uint8) for o in range(n)]
        try:
            _all_to_all_varlen(chunks, dist, torch.device("cpu"))
            q.put((rank, "ok"))
        except RuntimeError as e:
            q.put((rank, "refused: " + str(e)))
    finally:
        dist.destroy_process_group()


def test_all_to_all_refuses_on_every_rank_gloo():
    """A rank with a malformed exchange raises on EVERY rank (multi.agree) instead of leaving the
    others blocked in the collective (fail loudly, not hang)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_a2a_bad_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    assert all(v.startswith("refused") for v in got.values()), got
