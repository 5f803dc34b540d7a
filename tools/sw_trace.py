"""Per-workgroup trace of k_sweep (a LDB_SW_TRACE build: LAZYDB_GPU_LIB=.../var_def_LDB_SW_TRACE_1.so): five
writer-mix files of MiB each, scanned as one batch (ldb_scan_files_dev; LDB_DEBUG=1 LDB_SWEEP_SPLIT=0/1 picks
one launch over (vg, n) or one per file) or one by one. Prints, per file, the stream span, the workgroups'
stream durations (median / p90 / max) and the link tail. usage: python tools/sw_trace.py batch|single [MiB]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from lazydb_amd import Engine, _native as N
from oracle import coracle   # input generator only

W = 8 * 1024


def main():
    mode = sys.argv[1]
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    eng = Engine(0)
    imgs = [coracle.gen_writer_log(mib << 20, 50 + i)[0] for i in range(5)]
    k = len(imgs)
    d = [torch.from_numpy(im).cuda() for im in imgs]
    caps = [im.size // 32 for im in imgs]
    outs = [eng.alloc_out(c) for c in caps]
    res = torch.zeros(N.RESULT_BYTES * k, dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.current_stream()
    args = (eng.ctx, k, (C.c_void_p * k)(*[x.data_ptr() for x in d]), (C.c_uint64 * k)(*[im.size for im in imgs]),
            (C.c_uint32 * k)(*range(1, k + 1)), N.FILEIO, N.TUPLE_INDEX, (C.c_void_p * k)(*[o.data_ptr() for o in outs]),
            (C.c_uint64 * k)(*caps), C.c_void_p(res.data_ptr()), C.c_void_p(s.cuda_stream))
    rbuf = eng.alloc_result()

    def once():
        if mode == "batch":
            N.check(N.lib().ldb_scan_files_dev(*args), "ldb_scan_files_dev")
        else:
            for i in range(k):
                eng.scan_dev_async(d[i], fid=i + 1, out=outs[i], cap=caps[i], result=rbuf)

    for _ in range(3):
        once()
    torch.cuda.synchronize()
    tr = np.zeros(W * 4, dtype=np.uint64)
    N.lib().ldb_debug_swtrace(tr.ctypes.data_as(C.c_void_p), 1)
    once()
    torch.cuda.synchronize()
    N.check(N.lib().ldb_debug_swtrace(tr.ctypes.data_as(C.c_void_p), 0), "ldb_debug_swtrace")
    t = tr.reshape(W, 4).astype(np.int64)
    used = t[:, 0] != 0
    t0 = t[used, 0].min()
    g = int(used.sum()) // k
    print(f"{mode}: {k} files x {mib} MiB, {g} workgroups per file (times in us from the first start)")
    for f in range(k):
        r = t[f * g:(f + 1) * g]
        st, se = (r[:, 0] - t0) / 100.0, (r[:, 1] - t0) / 100.0
        dur = se - st
        le = (r[:, 2].max() - t0) / 100.0
        print(f"  file {f + 1}: starts {st.min():7.1f}..{st.max():7.1f}  streams end {se.min():7.1f}..{se.max():7.1f}"
              f"  per-wg {np.median(dur):6.1f} / {np.percentile(dur, 90):6.1f} / {dur.max():6.1f}  link end {le:7.1f}"
              f" (tail {le - se.max():5.1f})  CUs {len(set(r[:, 3].tolist()))}")
    eng.close()


if __name__ == "__main__":
    main()
