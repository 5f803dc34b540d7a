"""GPU tests of the C-ABI's calling contract (include/lazydb_gpu.h), against the C oracle.

* ldb_scan_files_dev, the batch export: several files of one value type back to back on one stream.
* The threading contract of index.go:103-108: the reference replays the five value types from five
  goroutines at once, each walking its own fids in ascending order. Here five host threads each own
  an ldb_ctx and a HIP stream and scan their files concurrently (ctypes releases the GIL).
* One context used from two streams without a host synchronisation in between: the workspace fence
  (ldb_ctx::ws_ev) must order the two pipelines.
* ldb_host_register: the page-locked host-image path of ldb_scan_file.
* A fresh context's first merge right after large, dirty allocations were released to the driver:
  the sequence of DESIGN.md §7a.
"""
import ctypes as C
import threading

import numpy as np
import pytest

from oracle import coracle

pytestmark = pytest.mark.gpu


def to_dev(img):
    import torch
    return torch.from_numpy(np.ascontiguousarray(img, dtype=np.uint8)).to("cuda:0")


def same(res, tup, ref, rt):
    assert (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries), \
        (res.as_dict(), (ref.status, ref.end_off, ref.n_entries))
    assert tup.tobytes() == rt.tobytes()


def _files(seed, n):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        shape = i % 3
        if shape == 0:
            img = coracle.gen_log(int(rng.integers(1 << 20, 6 << 20)), seed * 10 + i, ksize=64, vsize=256)[0]
        elif shape == 1:
            img = coracle.gen_log(int(rng.integers(1 << 20, 4 << 20)), seed * 10 + i, ksize=64, value_mode=1,
                                  zipf_max=512)[0]
        else:
            img = coracle.gen_log(int(rng.integers(200_000, 1 << 20)), seed * 10 + i, ksize=16, vsize=40)[0]
        if i == n - 1:   # the last file carries a corrupt byte: ErrInvalidCrc mid-file
            img = img.copy()
            img[img.size // 2] ^= 0x11
        out.append(img)
    return out


def test_scan_files_dev_batch(gpu_engine):
    import torch
    from lazydb_amd import _native as N
    eng = gpu_engine
    imgs = _files(1, 6)
    d = [to_dev(im) for im in imgs]
    caps = [im.size // 10 + 16 for im in imgs]
    outs = [eng.alloc_out(c) for c in caps]
    res = torch.zeros(N.RESULT_BYTES * len(imgs), dtype=torch.uint8, device="cuda:0")
    k = len(imgs)
    ptrs = (C.c_void_p * k)(*[x.data_ptr() for x in d])
    lens = (C.c_uint64 * k)(*[im.size for im in imgs])
    fids = (C.c_uint32 * k)(*[5 + i for i in range(k)])
    optr = (C.c_void_p * k)(*[o.data_ptr() for o in outs])
    capa = (C.c_uint64 * k)(*caps)
    s = torch.cuda.current_stream()
    N.check(N.lib().ldb_scan_files_dev(eng.ctx, k, ptrs, lens, fids, N.FILEIO, N.TUPLE_INDEX, optr, capa,
                                       C.c_void_p(res.data_ptr()), C.c_void_p(s.cuda_stream)), "ldb_scan_files_dev")
    rb = res.cpu().numpy().tobytes()
    for i, im in enumerate(imgs):
        r = N.ScanResult.from_buffer_copy(rb[i * N.RESULT_BYTES:(i + 1) * N.RESULT_BYTES])
        assert r.fid == 5 + i
        n = min(r.n_entries, caps[i])
        tup = np.frombuffer(outs[i][: n * 16].cpu().numpy().tobytes(), N.INDEX_TUPLE)
        same(r, tup, *coracle.scan(im, 0))


def _scan_files(eng, imgs, io, kind, caps, fid0=5):
    """ldb_scan_files_dev over device copies of imgs; returns [(result, tuples)]"""
    import torch
    from lazydb_amd import _native as N
    dt = N.INDEX_TUPLE if kind == N.TUPLE_INDEX else N.ENTRY_TUPLE
    d = [to_dev(im) if im.size else to_dev(np.zeros(16, np.uint8)) for im in imgs]
    outs = [eng.alloc_out(max(c, 1), kind) for c in caps]
    res = torch.zeros(N.RESULT_BYTES * len(imgs), dtype=torch.uint8, device="cuda:0")
    k = len(imgs)
    s = torch.cuda.current_stream()
    N.check(N.lib().ldb_scan_files_dev(
        eng.ctx, k, (C.c_void_p * k)(*[x.data_ptr() for x in d]), (C.c_uint64 * k)(*[im.size for im in imgs]),
        (C.c_uint32 * k)(*[fid0 + i for i in range(k)]), io, kind, (C.c_void_p * k)(*[o.data_ptr() for o in outs]),
        (C.c_uint64 * k)(*caps), C.c_void_p(res.data_ptr()), C.c_void_p(s.cuda_stream)), "ldb_scan_files_dev")
    rb = res.cpu().numpy().tobytes()
    got = []
    for i in range(k):
        r = N.ScanResult.from_buffer_copy(rb[i * N.RESULT_BYTES:(i + 1) * N.RESULT_BYTES])
        n = min(r.n_entries, caps[i])
        got.append((r, np.frombuffer(outs[i].cpu().numpy().tobytes()[: n * dt.itemsize], dt)))
    return got


@pytest.mark.parametrize("io", [0, 1])
@pytest.mark.parametrize("kind", [0, 1])
def test_scan_files_dev_batched_pipeline(gpu_engine, golden, io, kind):
    """The batched pipeline (every stage one launch, grid.y = file): every golden fixture that is at
    least one header window long, plus run / Zipf / small-entry images of different lengths and one
    undersized output, scanned as ONE batch; each file must match its own oracle scan. A set holding
    a shorter image goes file by file (the same results)."""
    meta, gimgs = golden
    names = sorted({m["name"] for m in meta})
    imgs = [np.frombuffer(gimgs[nm], np.uint8) for nm in names]
    imgs = [im for im in imgs if im.size >= 38] + _files(7, 5)
    caps = [im.size // 10 + 16 for im in imgs]
    caps[-2] = 3   # LDB_ERR_CAPACITY for this file only
    for i, (r, tup) in enumerate(_scan_files(gpu_engine, imgs, io, kind, caps)):
        assert r.fid == 5 + i
        ref, rt = coracle.scan(imgs[i], io, fid=5 + i, tuple_kind=kind, cap=caps[i])
        assert (r.status, r.end_off, r.n_entries) == (ref.status, ref.end_off, ref.n_entries), (i, r.as_dict())
        assert tup.tobytes() == rt.tobytes(), i
    short = [np.frombuffer(gimgs[nm], np.uint8) for nm in names if len(gimgs[nm]) < 38][:3]
    mixed = short + _files(8, 2)
    for i, (r, tup) in enumerate(_scan_files(gpu_engine, mixed, io, kind, [im.size // 10 + 16 for im in mixed])):
        ref, rt = coracle.scan(mixed[i], io, fid=5 + i, tuple_kind=kind)
        assert (r.status, r.end_off, r.n_entries) == (ref.status, ref.end_off, ref.n_entries), (i, r.as_dict())
        assert tup.tobytes() == rt.tobytes(), i


def test_bytes_past_len_ignored(gpu_engine):
    """include/lazydb_gpu.h: the kernels may load up to 15 bytes past `len` (whole 16-B granules);
    those bytes must never change a result. Each image sits at the start of a larger device buffer
    whose bytes past `len` are random, 0x00 or 0xFF; cut lengths cover every residue mod 16, cuts
    inside an entry and on entry boundaries, for the run prefix (equal-sized entries) and the
    region pipeline (Zipf values), both IO rules."""
    import torch
    eng = gpu_engine
    run = coracle.gen_log(3 << 20, 51, ksize=64, vsize=256)
    zipf = coracle.gen_log(3 << 20, 52, ksize=64, value_mode=1, zipf_max=512)
    rng = np.random.default_rng(53)
    for img, n, end in (run, zipf):
        cuts = [end - 16 * 40 + r for r in range(16)] + [end, end - 1, end // 2 + 7, 4096 + 3]
        for fill in ("rand", 0x00, 0xFF):
            buf = rng.integers(0, 256, img.size + 64, dtype=np.uint8) if fill == "rand" else \
                np.full(img.size + 64, fill, np.uint8)
            for cut in cuts:
                host = buf.copy()
                host[:cut] = img[:cut]
                d = to_dev(host)
                for io in (0, 1):
                    res, tup = eng.scan_dev(d[:cut], io_type=io)   # a view: the poisoned bytes follow it
                    ref, rt = coracle.scan(np.ascontiguousarray(img[:cut]), io)
                    same(res, tup, ref, rt)


def test_scan_host_chunked_run_prefix(gpu_engine):
    """ldb_scan_file stages the image in 64 MiB chunks and runs the run prefix chunk by chunk as they
    land (ChunkPlan): runs that span chunks, a corrupt entry two chunks in, a run that ends mid-chunk
    and is followed by other entries, and Zipf values (no run); pageable and page-locked images,
    staged and in-place (LDB_DIRECT_IMAGE) reads."""
    import os
    eng = gpu_engine
    run = coracle.gen_log(150 << 20, 61, ksize=64, vsize=256)[0]
    bad = run.copy()
    bad[(100 << 20) + 77] ^= 0x02
    mixed = np.concatenate([run[: (90 << 20) // 332 * 332],
                            coracle.gen_log(40 << 20, 62, ksize=16, vsize=40)[0]])
    zipf = coracle.gen_log(130 << 20, 63, ksize=64, value_mode=1, zipf_max=2048)[0]
    for img in (run, bad, mixed, zipf):
        ref = coracle.scan(img, 0, fid=3)
        res, tup = eng.scan_host(img, fid=3)
        same(res, tup, *ref)
        eng.host_register(img)
        try:
            for direct in (False, True):
                if direct:   # (the library reads its switches only under LDB_DEBUG)
                    os.environ["LDB_DEBUG"] = "1"
                    os.environ["LDB_DIRECT_IMAGE"] = "1"
                try:
                    res, tup = eng.scan_host(img, fid=3)
                finally:
                    os.environ.pop("LDB_DIRECT_IMAGE", None)
                    os.environ.pop("LDB_DEBUG", None)
                same(res, tup, *ref)
        finally:
            eng.host_unregister(img)


def test_five_contexts_five_threads():
    """index.go:103-108: one replay per value type, concurrently; each thread owns a context and a
    stream and scans its fids in ascending order (index.go:68)."""
    import torch
    from lazydb_amd import Engine
    from lazydb_amd import _native as N
    types = 5
    per = [_files(100 + t, 3) for t in range(types)]
    dev = [[to_dev(im) for im in fl] for fl in per]
    engines = [Engine(0) for _ in range(types)]
    streams = [torch.cuda.Stream() for _ in range(types)]
    got = [[None] * 3 for _ in range(types)]
    errs = []
    start = threading.Barrier(types)

    def replay(t):
        try:
            eng, s = engines[t], streams[t]
            outs = []
            start.wait()
            for i, d in enumerate(dev[t]):
                cap = d.numel() // 10 + 16
                with torch.cuda.stream(s):   # the result's zero fill ordered before the scan on s
                    out = eng.alloc_out(cap)
                    res = eng.alloc_result()
                rc = N.lib().ldb_scan_file_dev(eng.ctx, C.c_void_p(d.data_ptr()), d.numel(), i + 1, N.FILEIO,
                                               N.TUPLE_INDEX, C.c_void_p(out.data_ptr()), cap,
                                               C.c_void_p(res.data_ptr()), C.c_void_p(s.cuda_stream))
                N.check(rc, "ldb_scan_file_dev")
                outs.append((out, res, cap))
            s.synchronize()
            for i, (out, res, cap) in enumerate(outs):
                r = N.ScanResult.from_buffer_copy(res.cpu().numpy().tobytes())
                n = min(r.n_entries, cap)
                got[t][i] = (r, np.frombuffer(out[: n * 16].cpu().numpy().tobytes(), N.INDEX_TUPLE))
        except Exception as e:   # surfaced below
            errs.append(e)

    ths = [threading.Thread(target=replay, args=(t,)) for t in range(types)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errs, errs
    for t in range(types):
        for i, im in enumerate(per[t]):
            same(*got[t][i], *coracle.scan(im, 0))
    for e in engines:
        e.close()


def test_one_context_two_streams_no_host_sync(gpu_engine):
    """Pipeline A (a large file) on stream 1, then pipeline B on stream 2 of the same context with no
    host synchronisation: B must wait for A's use of the shared workspace."""
    import torch
    from lazydb_amd import _native as N
    eng = gpu_engine
    a = coracle.gen_log(256 << 20, 31, ksize=64, vsize=256)[0]
    b = coracle.gen_log(3 << 20, 32, ksize=16, vsize=100)[0]
    da, db = to_dev(a), to_dev(b)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    oa, ob = eng.alloc_out(a.size // 300 + 16), eng.alloc_out(b.size // 10 + 16)
    ra, rb = eng.alloc_result(), eng.alloc_result()
    torch.cuda.synchronize()
    for _ in range(3):
        eng.scan_dev_async(da, out=oa, cap=a.size // 300 + 16, result=ra, stream=s1)
        eng.scan_dev_async(db, out=ob, cap=b.size // 10 + 16, result=rb, stream=s2)
    torch.cuda.synchronize()
    for d_out, d_res, cap, im in ((oa, ra, a.size // 300 + 16, a), (ob, rb, b.size // 10 + 16, b)):
        r = N.ScanResult.from_buffer_copy(d_res.cpu().numpy().tobytes())
        n = min(r.n_entries, cap)
        same(r, np.frombuffer(d_out[: n * 16].cpu().numpy().tobytes(), N.INDEX_TUPLE), *coracle.scan(im, 0))


def test_host_register_path(gpu_engine):
    """ldb_scan_file on a page-locked image scans it in place over PCIe (no staging copy, region
    pipeline only); on pageable memory it stages the image in chunks over the copy streams. Both
    against the oracle: equal-sized entries, Zipf values, a corrupt entry, both IO rules and tuple
    kinds; an unaligned-length image (its last 16-B granule lies partly past len)."""
    eng = gpu_engine
    imgs = [coracle.gen_log(32 << 20, 41, ksize=64, vsize=256)[0],
            coracle.gen_log(24 << 20, 42, ksize=64, value_mode=1, zipf_max=1024)[0]]
    bad = imgs[1].copy()
    bad[bad.size // 3] ^= 0x21
    imgs += [bad, imgs[0][: (16 << 20) + 13].copy()]
    for img in imgs:
        eng.host_register(img)
        try:
            for kind in (0, 1):
                for io in (0, 1):
                    res, tup = eng.scan_host(img, fid=7, io_type=io, kind=kind)
                    same(res, tup, *coracle.scan(img, io, fid=7, tuple_kind=kind))
        finally:
            eng.host_unregister(img)
        res, tup = eng.scan_host(img, fid=7)
        same(res, tup, *coracle.scan(img, 0, fid=7))
        # a page-locked tuple array is written in place (with the image staged, then in place too)
        from lazydb_amd import _native as N
        hout = np.zeros(img.size // 10 + 16, dtype=N.INDEX_TUPLE)
        eng.host_register(hout)
        try:
            res, tup = eng.scan_host(img, fid=7, out=hout)
            same(res, tup, *coracle.scan(img, 0, fid=7))
            eng.host_register(img)
            try:
                hout[:] = np.zeros(1, dtype=N.INDEX_TUPLE)
                res, tup = eng.scan_host(img, fid=7, io_type=1, out=hout)
                same(res, tup, *coracle.scan(img, 1, fid=7))
            finally:
                eng.host_unregister(img)
        finally:
            eng.host_unregister(hout)
        # registered for fewer bytes than cap tuples: staged and copied back, never written in place
        # past the registration
        half = hout[: hout.size // 2]
        eng.host_register(half)
        try:
            hout[:] = np.zeros(1, dtype=N.INDEX_TUPLE)
            res, tup = eng.scan_host(img, fid=7, out=hout)
            same(res, tup, *coracle.scan(img, 0, fid=7))
        finally:
            eng.host_unregister(half)


def test_fresh_context_first_merge_after_dirty_release():
    """DESIGN.md §7a's sequence: large allocations filled with non-zero bytes are freed back to the
    driver, then a new context's first merge (two contexts on two streams inside) must be exact."""
    import torch
    from lazydb_amd import Engine
    from tests import merge_cases as MC
    for cycle in range(3):
        junk = torch.full((3 << 30,), 0xA5, dtype=torch.uint8, device="cuda:0")
        del junk
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        eng = Engine(0)
        files, kw = MC.small_cases()["gen1"]
        d = [(to_dev(f[0]), f[1], f[2]) for f in files]
        out = eng.merge_dev(d, kw["active_fid"], kw["active_off"], kw["max_file_size"], kw["now"])
        ref, stream, pos, segs, live, stats = coracle.merge(files, kw["active_fid"], kw["active_off"],
                                                            kw["max_file_size"], kw["now"])
        assert out["result"].status == ref.status == 0
        assert out["stream"].cpu().numpy().tobytes() == stream.tobytes()
        assert out["pos"].tobytes() == pos.tobytes()
        torch.cuda.synchronize()
        eng.close()
