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


def merge_distributed(eng, files, max_fid: int, active_fid: int, active_off: int, max_file_size: int, now: int,
                      io_type: int = N.FILEIO, fetch_pos: bool = True):
    """Config 5 over the ranks of torch.distributed: this rank's contiguous fid block `files`
    ([(device tensor, fid, is_target)], ascending; blocks ascending in rank order); max_fid = the
    largest fid over all ranks. Returns this rank's piece: stream, positions, segments, liveness,
    per-file stats, start/end (fid, offset) of the global rollover chain."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
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


def merge_distributed_single(eng, files, active_fid: int, active_off: int, max_file_size: int, now: int,
                             io_type: int = N.FILEIO, fetch_pos: bool = True):
    """merge_distributed at world size 1 without torch.distributed: the plain merge, same outputs."""
    part = rank_merge(eng, files, [], 0, active_fid, active_off, max_file_size, now, io_type)
    pl = rank_place(eng, part, None, active_fid, active_off, max_file_size, fetch_pos)
    pl.update(stream=part["stream"], live=part["live"], stats=part["stats"], n_emit=part["n_emit"])
    return pl
