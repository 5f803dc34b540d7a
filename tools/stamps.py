"""Phase breakdown of k_scan_main from an LDB_STAMPS build (s_memtime per wave, summed)."""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from lazydb_amd import Engine, _native as N
from oracle import coracle

cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
cfg = cfg if cfg == "w" else int(cfg)
if cfg == "w":   # the writer-realistic mix (bench.py leg w)
    img, n, end = coracle.gen_writer_log(1 << 30, 30)
elif cfg == 3:
    img, n, end = coracle.gen_log(8 << 30, 2, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
else:
    img, n, end = coracle.gen_log(1 << 30, 1, ksize=64, vsize=256)
eng = Engine(0)
d = torch.from_numpy(img).cuda()
res, tup = eng.scan_dev(d)
L = N.lib()
L.ldb_debug_stamps.argtypes = [C.c_void_p, C.c_int]
buf = np.zeros(18, np.uint64)
L.ldb_debug_stamps(buf.ctypes.data, 1)
for _ in range(3):
    eng.scan_dev(d)
L.ldb_debug_stamps(buf.ctypes.data, 1)
names = ["setup", "walk#1", "link+repair", "folds", "summary", "emit", "dma_wait", "tail", "crc_pass", "-",
         "ch:decode", "ch:links", "ch:rewrite", "ch:crc", "ch:scan+chk", "ch:emit+sum", "ch:covered", "-"]
nreg = (img.size + 5119) // 5120
tot = buf.sum()
for k in range(17):
    print(f"{names[k]:20s} {buf[k] / (3 * nreg):10.0f} cyc/region  {100 * buf[k] / tot:5.1f}%")
print("status", res.status, "repairs", res.n_repairs)
