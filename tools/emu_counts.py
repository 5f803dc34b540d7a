"""Per-region SIMT cost model from the instrumented CPU emulator: for each counted event, the
average count per lane and the average per-region maximum over lanes (what a wavefront pays).
Build: make -C tests/emu _build/libldb_emu_cnt.so"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import coracle  # noqa: E402

L = C.CDLL(os.path.join(ROOT, "tests/emu/_build/libldb_emu_cnt.so"))
L.emu_scan.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_void_p, C.c_uint64,
                       C.POINTER(coracle.ScanResult), C.c_void_p]
L.emu_counters.argtypes = [C.c_void_p]
names = ["spec classify", "walk classify", "in-slice entry crc", "slow decode", "ev4"]
cases = {"cfg2 64/256": dict(ksize=64, vsize=256),
         "zipf s=1.1 max 4096": dict(ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096),
         "small 16/16": dict(ksize=16, vsize=16)}
for name, kw in cases.items():
    img, n, end = coracle.gen_log(8 << 20, 7, **kw)
    out = np.zeros(n + 16, coracle.INDEX_TUPLE)
    res = coracle.ScanResult()
    st = np.zeros(2, np.uint32)
    L.emu_scan(img.ctypes.data, img.size, 0, 0, out.ctypes.data, n + 16, C.byref(res), st.ctypes.data)
    c = np.zeros(17, np.uint64)
    L.emu_counters(c.ctypes.data)
    R = int(c[16])
    print(f"== {name}: {R} region runs, {n} entries, repairs {st[1]}")
    for i, nm in enumerate(names):
        if c[i]:
            print(f"  {nm:22s} per lane {c[i] / R / 64:6.3f}   wave (max over lanes) {c[8 + i] / R:6.3f}")
