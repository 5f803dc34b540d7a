"""The Go binding's shape driven through ctypes on the GPU.

index.go:103-108 replays the five value types from five goroutines at once, and a context is not safe
for concurrent calls (include/lazydb_gpu.h). The binding hands contexts out from a pool keyed by nothing
thread-related (a Go channel of *gpuCtx; here a queue.Queue) and sizes each output slice exactly:
ldb_scan_file_count, then ldb_scan_copy_out into an array of n_entries tuples (logfile/log_file.go:116,
the per-entry tuples ReadLogEntry answers from). More threads than contexts, every result against the
C oracle's restatement of the replay.
"""
import ctypes as C
import queue
import threading

import numpy as np
import pytest

from lazydb_amd import _native as N
from oracle import coracle

pytestmark = pytest.mark.gpu


def _images():
    imgs = []
    for s in range(3):
        w, _, _ = coracle.gen_writer_log(2 << 20, 40 + s)
        imgs.append(w)
    z, _, _ = coracle.gen_log(4 << 20, 9, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
    imgs.append(z)
    f, _, _ = coracle.gen_log(3 << 20, 2, ksize=32, vsize=200)
    imgs.append(f)
    c = z.copy()
    c[(3 << 20) + 17] ^= 1   # a CRC failure mid-file
    imgs.append(c)
    imgs.append(np.zeros(4096, dtype=np.uint8))   # the sentinel at offset 0: no entry
    return imgs


def test_pool_count_copy_more_threads_than_contexts():
    L = N.lib()
    pool = queue.Queue()
    ctxs = []
    for _ in range(2):
        c = C.c_void_p()
        N.check(L.ldb_ctx_create(0, C.byref(c)), "ldb_ctx_create")
        ctxs.append(c)
        pool.put(c)
    imgs = _images()
    failures = []

    def work(t):
        try:
            for j in range(4):
                img = imgs[(t + j) % len(imgs)]
                io, kind = j & 1, (j >> 1) & 1
                ctx = pool.get()   # no thread identity: any free context
                try:
                    res = N.ScanResult()
                    N.check(L.ldb_scan_file_count(ctx, img.ctypes.data, img.size, t, io, kind, C.byref(res)), "count")
                    n = int(res.n_entries)
                    dt = coracle.INDEX_TUPLE if kind == 0 else coracle.ENTRY_TUPLE
                    out = np.empty(max(n, 1), dtype=dt)   # exactly the tuples produced
                    got = C.c_uint64()
                    N.check(L.ldb_scan_copy_out(ctx, out.ctypes.data, n, C.byref(got)), "copy_out")
                finally:
                    pool.put(ctx)
                ref, rt = coracle.scan(img, io_type=io, fid=t, tuple_kind=kind)
                if (res.status, res.end_off, res.n_entries) != (ref.status, ref.end_off, ref.n_entries) or got.value != n:
                    failures.append((t, j, res.as_dict(), ref.n_entries, got.value))
                elif n and out[:n].tobytes() != rt[:n].tobytes():
                    failures.append((t, j, "tuples differ"))
        except Exception as e:  # noqa: BLE001 -- reported below, on the main thread
            failures.append((t, repr(e)))

    threads = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    # the retained tuples belong to the last scan call only: after another scan, copy_out refuses
    c0 = ctxs[0]
    res = N.ScanResult()
    img = imgs[0]
    N.check(L.ldb_scan_file_count(c0, img.ctypes.data, img.size, 0, 0, 0, C.byref(res)), "count")
    out = np.empty(1, dtype=coracle.INDEX_TUPLE)
    N.check(L.ldb_scan_file(c0, img.ctypes.data, img.size, 0, 0, 0, out.ctypes.data, 1, C.byref(res)), "scan")
    got = C.c_uint64()
    assert L.ldb_scan_copy_out(c0, out.ctypes.data, 1, C.byref(got)) == N.ERR_ARG
    for c in ctxs:
        N.check(L.ldb_ctx_destroy(c), "ldb_ctx_destroy")
    assert not failures, failures[:5]
