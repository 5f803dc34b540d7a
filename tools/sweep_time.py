"""Time the sweep tier on one Zipf log (config 3's value mix): k_sweep and k_sweep_fin by HIP events, for the
library LAZYDB_GPU_LIB names (A/B and attribution builds: tools/build_variants.py def_LDB_SW_ABL=<bits> on a checkout of b0eb7f1).
usage: python tools/sweep_time.py [mib] [reps] [zipf|writer]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from lazydb_amd import Engine
    from oracle import coracle
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    kind = sys.argv[3] if len(sys.argv) > 3 else "zipf"
    if kind == "writer":   # bench leg w's log (gen_writer_log, seed 30)
        img, n, end = coracle.gen_writer_log(mib << 20, 30)
    else:
        img, n, end = coracle.gen_log(mib << 20, 11, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
    eng = Engine(0)
    d = torch.from_numpy(img).to("cuda:0")
    res, _ = eng.scan_dev(d, cap=n + 1024)
    out, rb = eng.alloc_out(n + 1024, 0), eng.alloc_result()
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.15:   # clocks up (DVFS)
        eng.scan_dev_async(d, out=out, cap=n + 1024, result=rb)
        torch.cuda.synchronize()
    import ctypes as C
    import numpy as np
    from lazydb_amd import _native as N
    L = N.lib()
    st = hasattr(L, "ldb_debug_swstamps")
    if st:
        L.ldb_debug_swstamps.argtypes = [C.c_void_p, C.c_int]
        buf = np.zeros(16, dtype=np.uint64)
        L.ldb_debug_swstamps(buf.ctypes.data, 1)
    eng.timing_split(1)
    for _ in range(reps):
        eng.scan_dev_async(d, out=out, cap=n + 1024, result=rb)
    torch.cuda.synchronize()
    sw, fin = eng.timing_sweep()
    u, mm, tot, k = eng.timing_split(0)
    lib = os.path.basename(os.environ.get("LAZYDB_GPU_LIB", "liblazydb_gpu.so"))
    print(f"{lib}: {mib} MiB n={n} status {res.status} sweep_n {res.n_sweep}: k_sweep {sw * 1e3:.1f} us "
          f"({end / sw / 1e9 * 1e3:.0f} GB/s) fin {fin * 1e3:.1f} us pipeline {tot * 1e3:.1f} us "
          f"({end / tot / 1e9 * 1e3:.0f} GB/s)", flush=True)
    if st:
        torch.cuda.synchronize()
        L.ldb_debug_swstamps(buf.ctypes.data, 1)
        nw = max(int(buf[8]), 1)
        names = ["setup", "load wait", "candidates", "crc+tree", "decode", "loop", "flush+walk", "links(last wg)"]
        print("  per wave and scan (kcycles): " + ", ".join(
            f"{names[k]} {buf[k] / (nw if k != 7 else reps) / 1e3:.1f}" for k in range(8)), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
