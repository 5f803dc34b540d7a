"""Host-side driver of the MI355X log-scan engine.

`Engine` owns one ldb_ctx (per device / per caller thread, like the reference's
one replay goroutine per value type, index.go:103-108) and scans log-file images
that live in HBM (torch uint8 tensors on a ROCm device) or in host memory.

PyTorch is only the device-memory / stream plumbing here: every byte of the scan
is done by the gfx950 kernels in liblazydb_gpu.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


PINNED_D2H_MIN = 1 << 20


def d2h_bytes(t) -> bytes:
    """Device uint8 tensor -> host bytes. Large downloads land in a pinned staging block from torch's
    pinned-memory cache (page-locked once, never unlocked while the process runs) rather than in a
    fresh pageable tensor that the runtime would have to lock and that is unmapped right after."""
    import torch
    n = int(t.numel())
    if n < PINNED_D2H_MIN:
        return t.cpu().numpy().tobytes()
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h.copy_(t)
    return h.numpy().tobytes()


class Engine:
    def __init__(self, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise N.LdbError("no ROCm GPU visible: the log-scan engine has no CPU path")
        self.torch = torch
        self.device = device
        self.ctx = C.c_void_p()
        N.check(N.lib().ldb_ctx_create(device, C.byref(self.ctx)), "ldb_ctx_create")

    def close(self):
        if self.ctx:
            N.lib().ldb_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, max_len: int):
        N.check(N.lib().ldb_ctx_reserve(self.ctx, max_len), "ldb_ctx_reserve")

    # ---------------------------------------------------------------- device-resident
    def alloc_out(self, cap: int, kind: int = N.TUPLE_INDEX):
        nbytes = cap * (16 if kind == N.TUPLE_INDEX else 48)
        return self.torch.empty(max(nbytes, 16), dtype=self.torch.uint8, device=f"cuda:{self.device}")

    def alloc_result(self):
        return self.torch.zeros(N.RESULT_BYTES, dtype=self.torch.uint8, device=f"cuda:{self.device}")

    def scan_dev_async(self, img, fid: int = 0, io_type: int = N.FILEIO, kind: int = N.TUPLE_INDEX, out=None,
                       cap: int = 0, result=None, serial: bool = False, stream=None):
        """Enqueue a scan of a device-resident uint8 tensor on `stream` (default: torch's current)."""
        t = self.torch
        assert img.dtype == t.uint8 and img.is_cuda and img.is_contiguous()
        if stream is None:
            stream = t.cuda.current_stream(img.device)
        fn = N.lib().ldb_scan_file_dev_serial if serial else N.lib().ldb_scan_file_dev
        rc = fn(self.ctx, C.c_void_p(img.data_ptr()), img.numel(), fid, io_type, kind,
                C.c_void_p(out.data_ptr()) if out is not None else None, cap,
                C.c_void_p(result.data_ptr()), C.c_void_p(stream.cuda_stream))
        N.check(rc, "ldb_scan_file_dev")

    def scan_dev(self, img, fid: int = 0, io_type: int = N.FILEIO, kind: int = N.TUPLE_INDEX, cap: int | None = None,
                 serial: bool = False):
        """Scan a device-resident image; returns (result dict, tuples as a numpy structured array)."""
        if cap is None:
            cap = img.numel() // 10 + 16
        out = self.alloc_out(cap, kind)
        res = self.alloc_result()
        self.scan_dev_async(img, fid, io_type, kind, out, cap, res, serial)
        r = N.ScanResult.from_buffer_copy(res.cpu().numpy().tobytes())
        n = min(r.n_entries, cap)
        dt = N.INDEX_TUPLE if kind == N.TUPLE_INDEX else N.ENTRY_TUPLE
        tuples = np.frombuffer(d2h_bytes(out[: n * dt.itemsize]), dtype=dt) if n else np.zeros(0, dt)
        return r, tuples

    # ---------------------------------------------------------------- host memory
    def scan_host(self, img: np.ndarray, fid: int = 0, io_type: int = N.FILEIO, kind: int = N.TUPLE_INDEX,
                  cap: int | None = None, out: np.ndarray | None = None):
        """ldb_scan_file on a host image. `out`: the caller's tuple array (e.g. page-locked with
        host_register, so the kernels write it in place); default a fresh one of `cap` tuples."""
        img = np.ascontiguousarray(img, dtype=np.uint8)
        dt = N.INDEX_TUPLE if kind == N.TUPLE_INDEX else N.ENTRY_TUPLE
        if out is not None:
            assert out.dtype == dt and out.flags.c_contiguous
            cap = out.size
        else:
            if cap is None:
                cap = img.size // 10 + 16
            out = np.zeros(max(cap, 1), dtype=dt)
        res = N.ScanResult()
        N.check(N.lib().ldb_scan_file(self.ctx, img.ctypes.data if img.size else None, img.size, fid, io_type, kind,
                                      out.ctypes.data, cap, C.byref(res)), "ldb_scan_file")
        return res, out[: min(res.n_entries, cap)]

    # ---------------------------------------------------------------- merge / GC
    def merge_dev(self, files, active_fid: int, active_off: int, max_file_size: int, now: int,
                  io_type: int = N.FILEIO, stream_cap: int | None = None, pos_cap: int | None = None,
                  seg_cap: int = 256, live_cap: int | None = None, want_live: bool = True, stream=None,
                  fetch_pos: bool = True, last=None):
        """Merge the target files of one value type (db.go:383-427 Merge + mergeStr + writeLogEntry).

        files: list of (device uint8 tensor, fid, is_target), ascending fid. Returns a dict with
        'result' (MergeResult), 'stream' (device tensor, the compacted bytes), 'pos' (ldb_merge_pos
        records, numpy), 'segments' (numpy), 'live' (device uint8 tensor, one flag per replayed record)
        and 'stats' (per-file numpy). Outputs that turn out too small are re-sized and the call repeated
        (LDB_ERR_CAPACITY reports the sizes needed). last: a device uint8 tensor, one "last record of
        its key" flag per replayed record resolved by the key owners (cross-GPU merge): then
        ldb_merge_apply_dev."""
        t = self.torch
        dev = f"cuda:{self.device}"
        arr = self._merge_files(files)
        tot_len = sum(img.numel() for img, _, _ in files)
        tgt_len = sum(img.numel() for img, _, tg in files if tg)
        stream_cap = tgt_len if stream_cap is None else stream_cap
        pos_cap = tgt_len // 64 + 1024 if pos_cap is None else pos_cap
        live_cap = tot_len // 64 + 1024 if live_cap is None else live_cap
        if stream is None:
            stream = t.cuda.current_stream(dev)
        for _attempt in range(2):
            d_stream = t.empty(max(stream_cap, 16), dtype=t.uint8, device=dev)
            d_pos = t.empty(max(pos_cap, 1) * N.MERGE_POS.itemsize, dtype=t.uint8, device=dev)
            d_live = t.empty(max(live_cap, 1), dtype=t.uint8, device=dev) if want_live else None
            segs = np.zeros(max(seg_cap, 1), dtype=N.MERGE_SEGMENT)
            stats = np.zeros(max(len(files), 1), dtype=N.MERGE_FILE_STAT)
            res = N.MergeResult()
            res.bad_file = -1   # an argument error returns before the library fills the result
            tail = (active_fid, active_off, max_file_size, now, d_stream.data_ptr(), stream_cap, d_pos.data_ptr(),
                    pos_cap, segs.ctypes.data, seg_cap, d_live.data_ptr() if want_live else None,
                    live_cap if want_live else 0, stats.ctypes.data, C.byref(res), C.c_void_p(stream.cuda_stream))
            if last is None:
                rc = N.lib().ldb_merge_files_dev(self.ctx, len(files), C.addressof(arr), io_type, *tail)
            else:
                assert last.dtype == t.uint8 and last.is_cuda
                rc = N.lib().ldb_merge_apply_dev(self.ctx, len(files), C.addressof(arr), io_type,
                                                 C.c_void_p(last.data_ptr()) if last.numel() else None, *tail)
            if rc != N.ERR_CAPACITY or res.bad_file >= 0:
                break
            stream_cap = max(stream_cap, res.emit_bytes)
            pos_cap = max(pos_cap, res.n_emit)
            seg_cap = max(seg_cap, res.n_segments)
            live_cap = max(live_cap, res.n_records)
        if rc not in (N.LDB_OK,) and res.bad_file < 0:
            N.check(rc, "ldb_merge_files_dev")
        npos = min(res.n_emit, pos_cap)
        if not fetch_pos:   # leave the positions on the device (bench)
            pos = d_pos[: npos * N.MERGE_POS.itemsize]
        else:
            pos = (np.frombuffer(d2h_bytes(d_pos[: npos * N.MERGE_POS.itemsize]), dtype=N.MERGE_POS)
                   if npos else np.zeros(0, N.MERGE_POS))
        return {"rc": rc, "result": res, "stream": d_stream[: res.emit_bytes],
                "pos": pos, "segments": segs[: min(res.n_segments, seg_cap)],
                "live": d_live[: res.n_records] if want_live else None, "stats": stats[: len(files)]}

    def _merge_files(self, files):
        t = self.torch
        arr = (N.MergeFile * max(len(files), 1))()
        for i, (img, fid, tg) in enumerate(files):
            assert img.dtype == t.uint8 and img.is_cuda and img.is_contiguous()
            arr[i].d_image = img.data_ptr() if img.numel() else None
            arr[i].len = img.numel()
            arr[i].fid = fid
            arr[i].is_target = 1 if tg else 0
        return arr

    def merge_route(self, files, n_owners: int, io_type: int = N.FILEIO, stream=None):
        """ldb_merge_route_dev: this rank's records routed to n_owners key owners. Returns dict(result,
        recs (device uint8, 24-B ldb_route_rec, grouped by owner), keys (device uint8, grouped by owner),
        counts (numpy: records per owner), key_bytes (numpy: key bytes per owner))."""
        t = self.torch
        dev = f"cuda:{self.device}"
        arr = self._merge_files(files)
        if stream is None:
            stream = t.cuda.current_stream(dev)
        rec_cap = sum(img.numel() for img, _, _ in files) // 16 + 1024
        key_cap = sum(img.numel() for img, _, _ in files) + 16 * rec_cap
        for _attempt in range(2):
            recs = t.empty(max(rec_cap, 1) * N.ROUTE_REC.itemsize, dtype=t.uint8, device=dev)
            keys = t.empty(max(key_cap, 16), dtype=t.uint8, device=dev)
            counts = np.zeros(2 * n_owners, dtype=np.uint64)
            res = N.MergeResult()
            res.bad_file = -1
            rc = N.lib().ldb_merge_route_dev(self.ctx, len(files), C.addressof(arr), io_type, n_owners,
                                             recs.data_ptr(), rec_cap, keys.data_ptr(), key_cap, counts.ctypes.data,
                                             C.byref(res), C.c_void_p(stream.cuda_stream))
            if rc != N.ERR_CAPACITY or res.bad_file >= 0:
                break
            rec_cap, key_cap = int(counts[:n_owners].sum()), int(counts[n_owners:].sum())
        if rc != N.LDB_OK and res.bad_file < 0:
            N.check(rc, "ldb_merge_route_dev")
        nr, nk = int(counts[:n_owners].sum()), int(counts[n_owners:].sum())
        return {"rc": rc, "result": res, "recs": recs[: nr * N.ROUTE_REC.itemsize], "keys": keys[:nk],
                "counts": counts[:n_owners].astype(np.int64), "key_bytes": counts[n_owners:].astype(np.int64)}

    def merge_resolve(self, recs, keys, ord_, stream=None):
        """ldb_merge_resolve_dev at a key owner: recs (device uint8, 24-B route records, key_off rebased
        into `keys`), keys (device uint8), ord_ (device int64: source rank << 32 | seq). Returns the
        device uint8 "last record of its key" flags."""
        t = self.torch
        dev = f"cuda:{self.device}"
        n = recs.numel() // N.ROUTE_REC.itemsize
        last = t.empty(max(n, 1), dtype=t.uint8, device=dev)
        if stream is None:
            stream = t.cuda.current_stream(dev)
        N.check(N.lib().ldb_merge_resolve_dev(self.ctx, n, recs.data_ptr() if n else None,
                                              keys.data_ptr() if keys.numel() else None,
                                              ord_.data_ptr() if n else None, last.data_ptr(),
                                              C.c_void_p(stream.cuda_stream)), "ldb_merge_resolve_dev")
        return last[:n]

    def encode_entries(self, items, blob, active_fid: int, active_off: int, max_file_size: int, seg_cap: int = 256,
                       stream=None):
        """Batch writeLogEntry (tx.go:156-206 commit loop; EncodeEntry log_entry.go:48-78 + the rollover
        of db.go:485). items: numpy ENCODE_ITEM array; blob: device uint8 tensor holding the keys and
        values. Returns dict(result, stream (device tensor), pos (numpy ldb_merge_pos), segments)."""
        t = self.torch
        dev = f"cuda:{self.device}"
        items = np.ascontiguousarray(items, dtype=N.ENCODE_ITEM)
        n = items.size
        d_items = t.from_numpy(items.view(np.uint8).reshape(-1).copy()).to(dev) if n else None
        cap = int(n * 38 + (int(items["k_size"].sum()) + int(items["v_size"].sum()) if n else 0)) + 16
        if stream is None:
            stream = t.cuda.current_stream(dev)
        for _attempt in range(2):
            d_stream = t.empty(max(cap, 16), dtype=t.uint8, device=dev)
            d_pos = t.empty(max(n, 1) * N.MERGE_POS.itemsize, dtype=t.uint8, device=dev)
            segs = np.zeros(max(seg_cap, 1), dtype=N.MERGE_SEGMENT)
            res = N.MergeResult()
            rc = N.lib().ldb_encode_entries_dev(
                self.ctx, n, d_items.data_ptr() if n else None, blob.data_ptr() if blob.numel() else None,
                active_fid, active_off, max_file_size, d_stream.data_ptr(), cap, d_pos.data_ptr(), n,
                segs.ctypes.data, seg_cap, C.byref(res), C.c_void_p(stream.cuda_stream))
            if rc != N.ERR_CAPACITY:
                break
            seg_cap = max(seg_cap, res.n_segments)
        N.check(rc, "ldb_encode_entries_dev")
        pos = (np.frombuffer(d2h_bytes(d_pos[: n * N.MERGE_POS.itemsize]), dtype=N.MERGE_POS)
               if n else np.zeros(0, N.MERGE_POS))
        return {"result": res, "stream": d_stream[: res.emit_bytes], "pos": pos,
                "segments": segs[: res.n_segments]}

    def encode_entries_dev(self, d_items, n: int, blob, cap: int, active_fid: int, active_off: int,
                           max_file_size: int, seg_cap: int = 256, stream=None):
        """encode_entries with the ENCODE_ITEM array already on the device (d_items: uint8 tensor of
        n * 48 bytes) and the stream capacity given (n * 38 + the key and value bytes suffice)."""
        t = self.torch
        dev = f"cuda:{self.device}"
        if stream is None:
            stream = t.cuda.current_stream(dev)
        for _attempt in range(2):
            d_stream = t.empty(max(cap, 16), dtype=t.uint8, device=dev)
            d_pos = t.empty(max(n, 1) * N.MERGE_POS.itemsize, dtype=t.uint8, device=dev)
            segs = np.zeros(max(seg_cap, 1), dtype=N.MERGE_SEGMENT)
            res = N.MergeResult()
            rc = N.lib().ldb_encode_entries_dev(
                self.ctx, n, d_items.data_ptr() if n else None, blob.data_ptr() if blob.numel() else None,
                active_fid, active_off, max_file_size, d_stream.data_ptr(), cap, d_pos.data_ptr(), n,
                segs.ctypes.data, seg_cap, C.byref(res), C.c_void_p(stream.cuda_stream))
            if rc != N.ERR_CAPACITY:
                break
            seg_cap = max(seg_cap, res.n_segments)
            cap = max(cap, res.emit_bytes)
        N.check(rc, "ldb_encode_entries_dev")
        return {"result": res, "stream": d_stream[: res.emit_bytes], "pos": d_pos[: n * N.MERGE_POS.itemsize],
                "segments": segs[: res.n_segments]}

    def merge_timing(self):
        a, b, c = C.c_double(), C.c_double(), C.c_double()
        N.check(N.lib().ldb_merge_timing(self.ctx, C.byref(a), C.byref(b), C.byref(c)), "merge_timing")
        return a.value, b.value, c.value

    def host_register(self, img: np.ndarray):
        """Page-lock a host image (ldb_host_register) so ldb_scan_file copies it by direct DMA."""
        N.check(N.lib().ldb_host_register(self.ctx, img.ctypes.data, img.nbytes), "ldb_host_register")

    def host_unregister(self, img: np.ndarray):
        N.check(N.lib().ldb_host_unregister(self.ctx, img.ctypes.data), "ldb_host_unregister")

    def read_ceiling(self, d_img, iters: int = 20) -> float:
        """GB/s of a read-only reduction over the device image (the practical HBM-read ceiling)."""
        g = C.c_double()
        N.check(N.lib().ldb_read_ceiling(self.ctx, d_img.data_ptr(), d_img.numel(), iters, C.byref(g)), "read_ceiling")
        return g.value

    def timing(self, enable: int = -1):
        a, b, n = C.c_double(), C.c_double(), C.c_uint64()
        N.check(N.lib().ldb_kernel_timing(self.ctx, enable, C.byref(a), C.byref(b), C.byref(n)), "timing")
        return a.value, b.value, n.value

    def timing_split(self, enable: int = -1):
        """(avg k_uniform ms, avg k_region ms, avg pipeline ms, launches) since the last reset."""
        u, a, b, n = C.c_double(), C.c_double(), C.c_double(), C.c_uint64()
        N.check(N.lib().ldb_kernel_timing_split(self.ctx, enable, C.byref(u), C.byref(a), C.byref(b), C.byref(n)),
                "timing_split")
        return u.value, a.value, b.value, n.value

    def timing_tail(self, n: int = 7):
        """Per-phase averages (ms, device clock) over the timed scans (ldb_kernel_timing_tail): [0] unused, [1] the
        sweep checks (k_region phase F), [2..6] regions, links, repair, cross-region CRCs, compaction (phases
        M, L, R, C, K)."""
        a = (C.c_double * n)()
        if not hasattr(N.lib(), "ldb_kernel_timing_tail"):   # an A/B build of an older revision
            return list(a)
        N.check(N.lib().ldb_kernel_timing_tail(self.ctx, a, n), "timing_tail")
        return list(a)

    def timing_sweep(self):
        """(avg k_sweep ms, avg phase-F ms) over the timed launches: the sweep tier's stream and its checks (query)."""
        a, b = C.c_double(), C.c_double()
        N.check(N.lib().ldb_kernel_timing_sweep(self.ctx, C.byref(a), C.byref(b)), "timing_sweep")
        return a.value, b.value
