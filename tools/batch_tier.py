"""The batched replay (ldb_scan_files_dev: index.go:103-108's five value types at once) through the sweep
tier: five Zipf-value logs (config 3's shape) and five writer-mix logs, each batch checked against the oracle
(status, end, count, every tuple, the tier's share), then timed beside the same files scanned one by one
(ldb_scan_file_dev). usage: python tools/batch_tier.py [MiB per file] [files per batch] [w: the writer mix only]"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from lazydb_amd import Engine, _native as N
from oracle import coracle   # checker only


def run(eng, name, imgs, reps=10):
    k = len(imgs)
    d = [torch.from_numpy(im).cuda() for im in imgs]
    refs = [coracle.scan(im, 0, fid=i + 1) for i, im in enumerate(imgs)]
    caps = [int(r[0].n_entries) + 1024 for r in refs]
    outs = [eng.alloc_out(c) for c in caps]
    res = torch.zeros(N.RESULT_BYTES * k, dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.current_stream()
    args = (eng.ctx, k, (C.c_void_p * k)(*[x.data_ptr() for x in d]), (C.c_uint64 * k)(*[im.size for im in imgs]),
            (C.c_uint32 * k)(*range(1, k + 1)), N.FILEIO, N.TUPLE_INDEX, (C.c_void_p * k)(*[o.data_ptr() for o in outs]),
            (C.c_uint64 * k)(*caps), C.c_void_p(res.data_ptr()), C.c_void_p(s.cuda_stream))
    N.check(N.lib().ldb_scan_files_dev(*args), "ldb_scan_files_dev")
    torch.cuda.synchronize()
    rb = res.cpu().numpy().tobytes()
    ok, nsw, nent, tot = True, 0, 0, 0
    for i in range(k):
        r = N.ScanResult.from_buffer_copy(rb[i * N.RESULT_BYTES:(i + 1) * N.RESULT_BYTES])
        ref, rt = refs[i]
        ok &= (r.status, r.end_off, r.n_entries) == (ref.status, ref.end_off, ref.n_entries) and \
            outs[i][: r.n_entries * 16].cpu().numpy().tobytes() == rt.tobytes()
        nsw += r.n_sweep
        nent += r.n_entries
        tot += r.end_off
    for _ in range(3):
        N.lib().ldb_scan_files_dev(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        N.lib().ldb_scan_files_dev(*args)
    torch.cuda.synchronize()
    ms_b = (time.perf_counter() - t0) * 1e3 / reps
    rbuf = eng.alloc_result()
    for _ in range(3):
        for i in range(k):
            eng.scan_dev_async(d[i], fid=i + 1, out=outs[i], cap=caps[i], result=rbuf)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        for i in range(k):
            eng.scan_dev_async(d[i], fid=i + 1, out=outs[i], cap=caps[i], result=rbuf)
    torch.cuda.synchronize()
    ms_s = (time.perf_counter() - t0) * 1e3 / reps
    print(f"{name}: {k} files, {tot / 2**30:.3f} GiB, {nent} entries, tier {nsw} ({nsw / max(1, nent):.3f}); batched "
          f"{ms_b:.3f} ms = {tot / (ms_b * 1e-3) / 2**30:.1f} GiB/s, one by one {ms_s:.3f} ms = "
          f"{tot / (ms_s * 1e-3) / 2**30:.1f} GiB/s; verified {ok}", flush=True)
    assert ok


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    nf = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    eng = Engine(0)
    if sys.argv[3:4] != ["w"]:
        run(eng, "Zipf values (config 3 shape)",
            [coracle.gen_log(mib << 20, 30 + i, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)[0] for i in range(nf)])
    run(eng, "writer mix", [coracle.gen_writer_log(mib << 20, 50 + i)[0] for i in range(nf)])
    eng.close()


if __name__ == "__main__":
    main()
