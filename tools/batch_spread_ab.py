"""the batched scan's grid spread (LDB_BATCH_SPREAD) on a batch that needs the region
pipeline -- 8 writer-mix files of 128 MiB (gen_writer_log: no run prefix covers them) scanned as one
ldb_scan_files_dev batch, checked against the oracle, then timed. The spread is read once per process:
run once per setting. usage: LDB_BATCH_SPREAD=0|1 python tools/batch_spread_ab.py"""
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

eng = Engine(0)
k = 8
imgs = [coracle.gen_writer_log(128 << 20, 40 + i)[0] for i in range(k)]
d = [torch.from_numpy(im).cuda() for im in imgs]
caps = [im.size // 16 + 16 for im in imgs]
outs = [eng.alloc_out(c) for c in caps]
res = torch.zeros(N.RESULT_BYTES * k, dtype=torch.uint8, device="cuda:0")
s = torch.cuda.current_stream()
args = (eng.ctx, k, (C.c_void_p * k)(*[x.data_ptr() for x in d]), (C.c_uint64 * k)(*[im.size for im in imgs]),
        (C.c_uint32 * k)(*range(1, k + 1)), N.FILEIO, N.TUPLE_INDEX, (C.c_void_p * k)(*[o.data_ptr() for o in outs]),
        (C.c_uint64 * k)(*caps), C.c_void_p(res.data_ptr()), C.c_void_p(s.cuda_stream))
N.check(N.lib().ldb_scan_files_dev(*args), "ldb_scan_files_dev")
torch.cuda.synchronize()
rb = res.cpu().numpy().tobytes()
ok = True
for i, im in enumerate(imgs):
    r = N.ScanResult.from_buffer_copy(rb[i * N.RESULT_BYTES:(i + 1) * N.RESULT_BYTES])
    ref, rt = coracle.scan(im, 0, fid=i + 1, cap=caps[i])
    n = min(r.n_entries, caps[i])
    ok &= (r.status, r.end_off, r.n_entries) == (ref.status, ref.end_off, ref.n_entries) and \
        outs[i][: n * 16].cpu().numpy().tobytes() == rt.tobytes()
for _ in range(3):
    N.lib().ldb_scan_files_dev(*args)
torch.cuda.synchronize()
reps = 10
t0 = time.perf_counter()
for _ in range(reps):
    N.lib().ldb_scan_files_dev(*args)
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1e3 / reps
tot = sum(int(N.ScanResult.from_buffer_copy(rb[i * N.RESULT_BYTES:(i + 1) * N.RESULT_BYTES]).end_off) for i in range(k))
print(f"LDB_BATCH_SPREAD={os.environ.get('LDB_BATCH_SPREAD', '(default 1)')}: {k} writer-mix files, "
      f"{tot / 2**30:.3f} GiB, {ms:.3f} ms/batch, {tot / (ms * 1e-3) / 2**30:.1f} GiB/s, verified {ok}")
eng.close()
