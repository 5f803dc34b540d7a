"""ldb_scan_file on a page-locked config-2 image and tuple array, a few times (for a rocprofv3
kernel + memory-copy trace of the e2e path)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from lazydb_amd import Engine, _native as N
from oracle import coracle

img, n, end = coracle.gen_log(1 << 30, 1, ksize=64, vsize=256)
eng = Engine(0)
hout = np.zeros(n + 1024, dtype=N.INDEX_TUPLE)
eng.host_register(img)
eng.host_register(hout)
for i in range(4):
    t0 = time.perf_counter()
    res, _ = eng.scan_host(img, fid=1, out=hout)
    print(f"iter {i}: {1e3 * (time.perf_counter() - t0):.2f} ms, n={res.n_entries}", flush=True)
eng.host_unregister(hout)
eng.host_unregister(img)
