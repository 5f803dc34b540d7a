"""k_uniform setup phases from an LDB_STAMPS build (tools/build_variants.py stamps): s_memtime cycles per
workgroup for the LP2 block and for uni_prepare. usage: LAZYDB_GPU_LIB=.../var_stamps.so python tools/uni_stamps.py [4s] [1] [2] [4]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from lazydb_amd import Engine, _native as N
from oracle import coracle

eng = Engine(0)
L = N.lib()
L.ldb_debug_stamps.argtypes = [C.c_void_p, C.c_int]
L.ldb_debug_ustamps.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(18, np.uint64)
ub = np.zeros(24, np.uint64)
PH = ["win0", "dec0+comb(+WG0 discovery)", "probes(WG0)", "decN(WG0)", "memo(WG0 x6)", "comb-rebuild", "verify(w0)", "fill", "finish", "wait", "rounds(WG0)", "round-time(WG0)", "publish(WG0)", "geometry(WG0 x6)", "probe-t0(WG0)", "barrier2(WG0)", "prep-decode(WG>0)", "prep-to-decoded(WG>0)", "prep-comb(WG>0)"]
def cases():
    want = sys.argv[1:] or ["4s", "1"]
    if "4s" in want:
        yield "cfg4-shape 64 MiB", coracle.gen_log(64 << 20, 1, ksize=64, vsize=256)
    if "1" in want:
        yield "cfg1 bench log", coracle.gen_bench_log(512 << 20, 1, n_entries=500_000)
    for c in ("2", "4"):
        if c in want:
            sys.argv = sys.argv[:1]
            import bench
            img, n, end, _, _ = bench.make_image(int(c), 0)
            yield f"cfg{c} bench image", (img, n, end)


for name, (img, n, end) in cases():
    d = torch.from_numpy(img).cuda()
    io = 1 if name.startswith("cfg1") else 0
    eng.scan_dev(d, io_type=io, cap=n + 16)
    torch.cuda.synchronize()
    L.ldb_debug_stamps(buf.ctypes.data, 1)
    L.ldb_debug_ustamps(ub.ctypes.data, 1)
    reps = 10
    for _ in range(reps):
        eng.scan_dev(d, io_type=io, cap=n + 16)
    torch.cuda.synchronize()
    L.ldb_debug_stamps(buf.ctypes.data, 1)
    L.ldb_debug_ustamps(ub.ctypes.data, 1)
    nwg = 256
    print(f"{name}: LP2 block {buf[9] / (reps * nwg):8.0f} cyc/WG, uni_prepare {buf[17] / (reps * nwg):8.0f} cyc/WG "
          f"(s_memtime counts shader clocks)")
    # WG0-only phases (discovery) per launch; the rest averaged over the workgroups
    print("   " + " ".join(f"{k} {ub[i] / (reps * (1 if 'WG0' in k and '+' not in k else (nwg - 1 if 'WG>0' in k else nwg))):.0f}" for i, k in enumerate(PH)))
