"""Cross-GPU merge/GC of one file set (BASELINE config 5 on N GPUs).

The reference merge (db.go:383-427, mergeStr db.go:243-265) keeps a record iff it is its key's final
index value after the replay of *every* file in (fid, offset) order (index.go:15-26, 68-95: Put per
record, Delete on SDelete), and appends the kept records of the target files to one writeLogEntry
rollover chain (db.go:473-523). With the files split over ranks in contiguous fid blocks (rank r
holds a block below rank r+1's), both couplings are one exchange each:

1. Liveness. A record of rank r is final for its key iff it is final within rank r's own block and
   no later rank's block holds its key. Each rank condenses its block into a *summary log*: its
   locally-final records plus every SDelete record, in (fid, offset) order, re-encoded as key-only
   LazyDB entries (stat kept, value empty) by the batch encoder (ldb_encode_entries_dev). Replaying
   such a summary leaves the same final state per key as replaying the block: a key whose final
   record is a Put ends present, one whose final record is an SDelete ends deleted. The summaries
   are all-gathered (RCCL over xGMI), and rank r runs the ordinary merge engine
   (ldb_merge_files_dev) on its own files followed by the summaries of ranks r+1.. as non-target
   files with fids above every real fid. Last-writer-wins over that list is exactly the global rule
   for rank r's records.
2. Placement. Each rank's compacted stream is one piece of the global stream, in rank order. The
   entry sizes are all-gathered; rank r re-runs the rollover over ranks 0..r-1's sizes from the
   active file's append offset to find where its piece starts (ldb_merge_repack_dev), then
   re-places its own records from there. Rollover is a greedy chain, so this is the serial
   writeLogEntry sequence exactly.

Every byte of scanning, hashing, liveness, encoding, packing and copying runs in the gfx950
kernels of liblazydb_gpu.so; this module only moves buffers between ranks. Phases are separate
functions so one process can play every rank (tests/test_gpu_cross_merge.py), and `merge_distributed`
wires them with torch.distributed.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N
from .engine import d2h_bytes

SUMMARY_PAD = 64          # zero bytes after a summary log: the replay stops at the zero sentinel
                          # (log_file.go:124-126) under both IOController bound rules
NO_ROLLOVER = 1 << 62     # summaries are one log each


def summary_fid_base(max_fid: int) -> int:
    """Fids given to summary logs: above every real fid, ascending in rank order."""
    return max_fid + 1


def rank_summary(eng, files, io_type: int = N.FILEIO):
    """Phase 1 on one rank. files: [(device uint8 tensor, fid, is_target)], ascending fid.
    Returns the summary log (device uint8 tensor, zero-padded) and its record count. Device-resident:
    the replay tuples, the selection and the ENCODE_ITEM array never leave the GPU."""
    t = eng.torch
    dev = f"cuda:{eng.device}"
    plain = [(img, fid, False) for img, fid, _ in files]
    # local last-writer-wins over this block alone (no target: the pre-resolution pass, f1)
    out = eng.merge_dev(plain, 0, 0, NO_ROLLOVER, 0, io_type=io_type, stream_cap=0, pos_cap=0, seg_cap=1)
    r = out["result"]
    if r.bad_file >= 0:
        raise N.LdbError(f"replay of file {files[r.bad_file][1]} failed: {N.status_str(r.status)}")
    live = out["live"]
    blob = t.cat([img for img, _, _ in files]) if len(files) > 1 else files[0][0]
    tups, ress = [], []
    for img, fid, _ in files:   # index tuples of every file, enqueued back to back
        cap = img.numel() // 10 + 16
        o, res = eng.alloc_out(cap), eng.alloc_result()
        eng.scan_dev_async(img, fid, io_type, N.TUPLE_INDEX, o, cap, res)
        tups.append(o)
        ress.append(res)
    counts = [N.ScanResult.from_buffer_copy(x.cpu().numpy().tobytes()).n_entries for x in ress]
    assert sum(counts) == r.n_records, (counts, r.n_records)
    sel, base, k = [], 0, 0
    for (img, _, _), o, n in zip(files, tups, counts):
        q = o[: 16 * n].view(t.int64).view(n, 2)                    # ldb_index_tuple: pos, k | v << 32
        pos, kv = q[:, 0], q[:, 1]
        stat = (pos >> 52) & 0xFF
        keep = (live[k:k + n] != 0) | (stat == 1)
        key_off = (pos & ((1 << 40) - 1)) + ((pos >> 40) & 0x3F) + base
        sel.append(t.stack([key_off, kv & 0xFFFFFFFF, stat], 1)[keep])
        base += img.numel()
        k += n
    sel = t.cat(sel) if sel else t.zeros(0, 3, dtype=t.int64, device=dev)
    m = int(sel.shape[0])
    items = t.zeros(m, 6, dtype=t.int64, device=dev)              # ENCODE_ITEM, 48 B
    items[:, 0] = sel[:, 0]                                       # key_off
    items[:, 1] = sel[:, 0]                                       # value_off (empty value)
    items[:, 2] = sel[:, 1]                                       # k_size, v_size = 0
    items[:, 5] = sel[:, 2] << 16                                 # tx_stat = 0, stat
    cap = m * 38 + int(sel[:, 1].sum().item()) + 16
    enc = eng.encode_entries_dev(items.view(t.uint8).view(-1), m, blob, cap, 0, 0, NO_ROLLOVER, seg_cap=4)
    s = enc["stream"]
    summ = t.zeros(s.numel() + SUMMARY_PAD, dtype=t.uint8, device=dev)
    summ[: s.numel()] = s
    return summ, m


def rank_merge(eng, files, later_summaries, sum_fid0: int, active_fid: int, active_off: int,
               max_file_size: int, now: int, io_type: int = N.FILEIO):
    """Phase 2 on one rank: the merge engine over its own files plus the later ranks' summaries
    (sum_fid0 + j for the j-th of them). The placement of the output is provisional (phase 3)."""
    allf = list(files) + [(s, sum_fid0 + j, False) for j, s in enumerate(later_summaries)]
    out = eng.merge_dev(allf, active_fid, active_off, max_file_size, now, io_type=io_type, fetch_pos=False)
    r = out["result"]
    if r.bad_file >= 0:
        raise N.LdbError(f"merge input {r.bad_file} failed: {N.status_str(r.status)}")
    nf = len(files)
    own_records = int(sum(int(x) for x in out["stats"]["n_entries"][:nf]))
    return {"result": r, "stream": out["stream"], "pos": out["pos"], "n_emit": r.n_emit,
            "live": out["live"][:own_records], "stats": out["stats"][:nf]}


def entry_sizes(eng, part):
    """Device uint32 entry sizes of a rank's emitted records, stream order (for the all-gather)."""
    t = eng.torch
    n = part["n_emit"]
    if n == 0:
        return t.zeros(0, dtype=t.int32, device=f"cuda:{eng.device}")
    return part["pos"].view(t.int32).view(n, 8)[:, 3].contiguous()   # ldb_merge_pos.entry_size


def repack(eng, n: int, d_sizes, d_pos, start_fid: int, start_off: int, max_file_size: int, seg_cap: int = 256):
    """ldb_merge_repack_dev: the rollover chain over n records from (start_fid, start_off)."""
    t = eng.torch
    stream = t.cuda.current_stream(f"cuda:{eng.device}")
    for _attempt in range(2):
        segs = np.zeros(max(seg_cap, 1), dtype=N.MERGE_SEGMENT)
        res = N.MergeResult()
        rc = N.lib().ldb_merge_repack_dev(
            eng.ctx, n, d_sizes.data_ptr() if (d_sizes is not None and n) else None,
            d_pos.data_ptr() if (d_pos is not None and n) else None, start_fid, start_off, max_file_size,
            segs.ctypes.data if seg_cap else None, seg_cap, C.byref(res), C.c_void_p(stream.cuda_stream))
        if rc != N.ERR_CAPACITY:
            break
        seg_cap = res.n_segments
    N.check(rc, "ldb_merge_repack_dev")
    return res, segs[: res.n_segments]


def rank_place(eng, part, earlier_sizes, active_fid: int, active_off: int, max_file_size: int,
               fetch_pos: bool = True):
    """Phase 3 on one rank: start state from the earlier ranks' entry sizes (rank order,
    concatenated, device int32), then this rank's records re-placed from it. Returns the start
    state, the segments (rank-local stream offsets), the end state and the positions (numpy)."""
    n_prev = int(earlier_sizes.numel()) if earlier_sizes is not None else 0
    st, _ = repack(eng, n_prev, earlier_sizes, None, active_fid, active_off, max_file_size, seg_cap=0) \
        if n_prev else (None, None)
    f0, o0 = (st.end_fid, st.end_off) if st is not None else (active_fid, active_off)
    n = part["n_emit"]
    res, segs = repack(eng, n, None, part["pos"], f0, o0, max_file_size)
    if not fetch_pos:   # leave the positions on the device (bench)
        pos = part["pos"]
    else:
        pos = (np.frombuffer(d2h_bytes(part["pos"]), dtype=N.MERGE_POS) if n
               else np.zeros(0, N.MERGE_POS))
    return {"start": (f0, o0), "end": (res.end_fid, res.end_off), "segments": segs, "pos": pos}


# --------------------------------------------------------------------------- hash-partitioned liveness
# The balanced form of coupling 1: instead of replaying the later ranks' summaries,
# every rank routes each of its records to the owner of its key (ldb_merge_route_dev: 24-B route
# record + key bytes, grouped by owner), one all-to-all delivers them, each owner resolves
# last-writer-wins over ~1/N of the keys by the global order (source rank, seq)
# (ldb_merge_resolve_dev), a second all-to-all returns one flag byte per record, and each rank merges
# its own files with those flags (ldb_merge_apply_dev). Per rank the device work is its own 1/N of the
# scans, of the hashing and of the table, whatever N.
ROUTE_REC_BYTES = N.ROUTE_REC.itemsize


def route_phase(eng, files, world: int, io_type: int = N.FILEIO):
    """Phase H1 on one rank: its records and keys grouped by owner. Returns the route dict of
    Engine.merge_route plus the per-owner byte splits of both buffers."""
    out = eng.merge_route(files, world, io_type)
    r = out["result"]
    if r.bad_file >= 0:
        raise N.LdbError(f"replay of file {files[r.bad_file][1]} failed: {N.status_str(r.status)}")
    out["rec_splits"] = [int(c) * ROUTE_REC_BYTES for c in out["counts"]]
    out["key_splits"] = [int(k) for k in out["key_bytes"]]
    return out


def owner_inputs(t, recv_recs, recv_keys, src_counts):
    """Owner side of the exchange: the route records and key blobs received from every source rank
    (rank order) joined into one array each; key offsets rebased into the joined blob; the global order
    ord = source rank << 32 | seq."""
    recs = t.cat(recv_recs) if recv_recs else None
    keys = t.cat(recv_keys) if recv_keys else None
    n = int(recs.numel()) // ROUTE_REC_BYTES if recs is not None else 0
    if n == 0:
        dev = recv_recs[0].device
        return t.zeros(0, dtype=t.uint8, device=dev), t.zeros(16, dtype=t.uint8, device=dev), \
            t.zeros(0, dtype=t.int64, device=dev)
    q = recs.view(t.int64).view(n, 3).clone()
    kb = t.tensor([0] + [int(k.numel()) for k in recv_keys[:-1]], dtype=t.int64, device=recs.device).cumsum(0)
    src = t.repeat_interleave(t.arange(len(src_counts), device=recs.device),
                              t.tensor(src_counts, dtype=t.int64, device=recs.device))
    q[:, 2] += kb[src]
    ord_ = (src.to(t.int64) << 32) | (q[:, 1] & 0xFFFFFFFF)
    if keys is None or keys.numel() == 0:
        # every received key is empty (pad16(0) = 0 bytes): the resolve still wants a key buffer
        keys = t.zeros(16, dtype=t.uint8, device=recs.device)
    return q.view(t.uint8).view(-1), keys, ord_


def last_by_seq(t, route, flags_from_owner, n_records: int):
    """Sender side of the return exchange: the owners' flags (owner order, each in the order the
    records were sent) scattered back to replay order."""
    dev = route["recs"].device
    last = t.zeros(max(n_records, 1), dtype=t.uint8, device=dev)
    n = int(route["recs"].numel()) // ROUTE_REC_BYTES
    if n:
        seq = route["recs"].view(t.int64).view(n, 3)[:, 1] & 0xFFFFFFFF
        last[seq] = t.cat(flags_from_owner)
    return last[:n_records]


def apply_phase(eng, files, last, active_fid: int, active_off: int, max_file_size: int, now: int,
                io_type: int = N.FILEIO):
    """Phase H3 on one rank: its own merge with the owners' liveness. Same output as rank_merge."""
    out = eng.merge_dev(files, active_fid, active_off, max_file_size, now, io_type=io_type, fetch_pos=False,
                        last=last)
    r = out["result"]
    if r.bad_file >= 0:
        raise N.LdbError(f"merge input {r.bad_file} failed: {N.status_str(r.status)}")
    return {"result": r, "stream": out["stream"], "pos": out["pos"], "n_emit": r.n_emit,
            "live": out["live"][: r.n_records], "stats": out["stats"][: len(files)]}


def hashed_sim(engs, blocks, active_fid: int, active_off: int, max_file_size: int, now: int,
               io_type: int = N.FILEIO, timer=None, fetch_pos: bool = True):
    """Every rank of the hash-partitioned merge in one process (tests, bench --xsim): engs[r] plays
    rank r (its own context), blocks[r] its files. The exchanges are slices. `timer(rank, phase, fn)`
    may wrap each rank's device phases. Returns the per-rank parts and places as merge_distributed."""
    t = engs[0].torch
    world = len(blocks)
    tm = timer or (lambda r, ph, fn: fn())
    routes = [tm(r, "route", lambda r=r: route_phase(engs[r], blocks[r], world, io_type)) for r in range(world)]
    flags = [[None] * world for _ in range(world)]   # flags[src][owner]
    for o in range(world):
        rr, kk, cnt = [], [], []
        for src in range(world):
            ro = routes[src]
            a = sum(ro["rec_splits"][:o])
            rr.append(ro["recs"][a: a + ro["rec_splits"][o]])
            ka = sum(ro["key_splits"][:o])
            kk.append(ro["keys"][ka: ka + ro["key_splits"][o]])
            cnt.append(int(ro["counts"][o]))
        recs, keys, ord_ = owner_inputs(t, rr, kk, cnt)
        last = tm(o, "resolve", lambda o=o, recs=recs, keys=keys, ord_=ord_: engs[o].merge_resolve(recs, keys, ord_))
        b = 0
        for src in range(world):
            flags[src][o] = last[b: b + cnt[src]]
            b += cnt[src]
    parts = []
    for r in range(world):
        lr = last_by_seq(t, routes[r], flags[r], int(routes[r]["result"].n_records))
        parts.append(tm(r, "apply", lambda r=r, lr=lr: apply_phase(engs[r], blocks[r], lr, active_fid, active_off,
                                                                    max_file_size, now, io_type)))
    sizes = [entry_sizes(engs[r], p) for r, p in enumerate(parts)]
    places = [tm(r, "place", lambda r=r: rank_place(engs[r], parts[r], t.cat(sizes[:r]) if r else None, active_fid,
                                                    active_off, max_file_size, fetch_pos)) for r in range(world)]
    return parts, places


# ---------------------------------------------------------------------------------- distributed
def _all_gather_varlen(x, dist):
    """All-gather 1-D tensors of different lengths (rank order). RCCL moves device tensors; gloo
    (CPU tests) is given host copies."""
    import torch
    world = dist.get_world_size()
    cpu = dist.get_backend() == "gloo"
    y = x.cpu() if cpu else x
    n = torch.tensor([y.numel()], dtype=torch.int64, device=y.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(v.item()) for v in ns]
    mx = max(max(ns), 1)
    send = torch.zeros(mx, dtype=y.dtype, device=y.device)
    send[: y.numel()] = y
    bufs = [torch.empty(mx, dtype=y.dtype, device=y.device) for _ in range(world)]
    dist.all_gather(bufs, send)
    return [b[:k].to(x.device) for b, k in zip(bufs, ns)]


def check_fid_blocks(files, dist, device=None):
    """Both cross-GPU merges take last-writer-wins order from the rank order (rank r's block below rank
    r+1's): a round-robin or misordered split would give wrong liveness silently, so it is refused.
    One all-gather of each rank's (fids ascending?, min fid, max fid); an empty block is skipped.
    Every rank raises on the same gathered values, so a bad block on one rank never leaves the others
    blocked in a later collective. `device`: where the collective buffer lives (the engine's GPU under
    RCCL; host memory under gloo), never taken from the files, which an empty block has none of."""
    import torch
    from .multi import coll_device
    dev = coll_device(device if device is not None else
                      (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"))
    fids = [int(f) for _, f, _ in files]
    ok = fids == sorted(fids) and len(set(fids)) == len(fids)
    mine = torch.tensor([1 if ok else 0] + ([min(fids), max(fids)] if fids else [-1, -1]), dtype=torch.int64,
                        device=dev)
    allb = [torch.zeros_like(mine) for _ in range(dist.get_world_size())]
    dist.all_gather(allb, mine)
    allb = [[int(v) for v in b.cpu()] for b in allb]
    bad = [r for r, b in enumerate(allb) if b[0] == 0]
    if bad:
        raise ValueError(f"rank(s) {bad}: fids not strictly ascending" + ("" if ok else f" (here: {fids})"))
    prev = None
    for r, (_, lo, hi) in enumerate(allb):
        if lo < 0:
            continue
        if prev is not None and lo <= prev:
            raise ValueError(f"fid blocks not ascending in rank order: rank {r} starts at fid {lo}, "
                             f"an earlier rank ends at {prev}")
        prev = hi


def merge_distributed(eng, files, max_fid: int, active_fid: int, active_off: int, max_file_size: int, now: int,
                      io_type: int = N.FILEIO, fetch_pos: bool = True):
    """Config 5 over the ranks of torch.distributed: this rank's contiguous fid block `files`
    ([(device tensor, fid, is_target)], ascending; blocks ascending in rank order); max_fid = the
    largest fid over all ranks. Returns this rank's piece: stream, positions, segments, liveness,
    per-file stats, start/end (fid, offset) of the global rollover chain."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    check_fid_blocks(files, dist, torch.device("cuda", eng.device))
    if world == 1:
        allsum = []
    else:   # rank r reads the summaries of ranks r+1..: nobody reads rank 0's
        summ = rank_summary(eng, files, io_type)[0] if rank > 0 else \
            torch.zeros(0, dtype=torch.uint8, device=files[0][0].device)
        allsum = _all_gather_varlen(summ, dist)
    part = rank_merge(eng, files, allsum[rank + 1:], summary_fid_base(max_fid) + rank + 1, active_fid, active_off,
                      max_file_size, now, io_type)
    sizes = _all_gather_varlen(entry_sizes(eng, part), dist) if world > 1 else []
    earlier = torch.cat(sizes[:rank]) if rank else None
    pl = rank_place(eng, part, earlier, active_fid, active_off, max_file_size, fetch_pos)
    pl.update(stream=part["stream"], live=part["live"], stats=part["stats"], n_emit=part["n_emit"])
    return pl


def _all_to_all_varlen(chunks, dist, device):
    """chunks[o] (1-D uint8 device tensors) to rank o; returns what every rank sent here, rank order.
    RCCL: all_to_all_single with the splits; gloo (CPU tests): an all-gather of everything, host copies.
    `device` is the engine's GPU (the collective's buffers follow the backend through coll_device), never
    taken from the chunks, which a refused call may not have. A rank with the wrong number of chunks makes
    every rank raise (multi.agree) before any byte moves."""
    import torch
    from .multi import agree, coll_device
    world = dist.get_world_size()
    rank = dist.get_rank()
    ok = len(chunks) == world and all(c.dtype == torch.uint8 and c.dim() == 1 for c in chunks)
    agree(ok, "all-to-all exchange", device)
    dev = coll_device(device)
    sizes = torch.tensor([int(c.numel()) for c in chunks], dtype=torch.int64)
    if dist.get_backend() == "gloo":
        flat = torch.cat(chunks).cpu() if chunks else torch.zeros(0, dtype=torch.uint8)
        allsz = [torch.zeros_like(sizes) for _ in range(world)]
        dist.all_gather(allsz, sizes)
        got = _all_gather_varlen(flat, dist)
        out = []
        for src in range(world):
            off = int(allsz[src][:rank].sum())
            out.append(got[src][off: off + int(allsz[src][rank])].to(device))
        return out
    sizes_d = sizes.to(dev)
    recv_sz = torch.empty_like(sizes_d)
    dist.all_to_all_single(recv_sz, sizes_d)
    recv_sz = [int(x) for x in recv_sz.cpu()]
    # the bytes sent and received over all ranks must balance: a transport or caller fault in the size
    # exchange makes every rank raise here, instead of posting inconsistent splits
    bal = torch.tensor([int(sizes.sum()) - sum(recv_sz)], dtype=torch.int64, device=dev)
    dist.all_reduce(bal)
    if int(bal.item()) != 0:
        raise RuntimeError(f"all-to-all exchange: sent and received byte totals differ by {int(bal.item())}")
    send = torch.cat(chunks) if chunks else torch.zeros(0, dtype=torch.uint8, device=dev)
    recv = torch.empty(sum(recv_sz), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(recv, send, output_split_sizes=recv_sz, input_split_sizes=[int(x) for x in sizes])
    out, b = [], 0
    for n in recv_sz:
        out.append(recv[b: b + n])
        b += n
    return out


def merge_hashed_distributed(eng, files, active_fid: int, active_off: int, max_file_size: int, now: int,
                             io_type: int = N.FILEIO, fetch_pos: bool = True):
    """The hash-partitioned cross-GPU merge over torch.distributed: route, one
    all-to-all of route records and keys, resolve at the owners, one all-to-all of flags back, apply,
    then the rollover chain as merge_distributed. Same return value."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    gdev = torch.device("cuda", eng.device)
    check_fid_blocks(files, dist, gdev)
    ro = route_phase(eng, files, world, io_type)
    rc = [ro["recs"][sum(ro["rec_splits"][:o]): sum(ro["rec_splits"][:o + 1])] for o in range(world)]
    kc = [ro["keys"][sum(ro["key_splits"][:o]): sum(ro["key_splits"][:o + 1])] for o in range(world)]
    got_r = _all_to_all_varlen(rc, dist, gdev)
    got_k = _all_to_all_varlen(kc, dist, gdev)
    recs, keys, ord_ = owner_inputs(torch, got_r, got_k, [int(x.numel()) // ROUTE_REC_BYTES for x in got_r])
    last = eng.merge_resolve(recs, keys, ord_)
    back, b = [], 0
    for x in got_r:
        n = int(x.numel()) // ROUTE_REC_BYTES
        back.append(last[b: b + n])
        b += n
    mine = _all_to_all_varlen(back, dist, gdev)
    lr = last_by_seq(torch, ro, mine, int(ro["result"].n_records))
    part = apply_phase(eng, files, lr, active_fid, active_off, max_file_size, now, io_type)
    sizes = _all_gather_varlen(entry_sizes(eng, part), dist) if world > 1 else []
    earlier = torch.cat(sizes[:rank]) if rank else None
    pl = rank_place(eng, part, earlier, active_fid, active_off, max_file_size, fetch_pos)
    pl.update(stream=part["stream"], live=part["live"], stats=part["stats"], n_emit=part["n_emit"])
    return pl


def merge_distributed_single(eng, files, active_fid: int, active_off: int, max_file_size: int, now: int,
                             io_type: int = N.FILEIO, fetch_pos: bool = True):
    """merge_distributed at world size 1 without torch.distributed: the plain merge, same outputs."""
    part = rank_merge(eng, files, [], 0, active_fid, active_off, max_file_size, now, io_type)
    pl = rank_place(eng, part, None, active_fid, active_off, max_file_size, fetch_pos)
    pl.update(stream=part["stream"], live=part["live"], stats=part["stats"], n_emit=part["n_emit"])
    return pl
