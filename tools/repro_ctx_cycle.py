"""Narrow down DESIGN.md §7a: create an engine, use one entry point, destroy it, repeat, and check
that plain host-to-device copies still work after each cycle. Modes: scan, host (ldb_scan_file),
merge (two contexts and two streams inside), encode. Prints one line per cycle; stops at the
first failure."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from lazydb_amd import Engine  # noqa: E402
from oracle import coracle  # noqa: E402
from tests import merge_cases as MC  # noqa: E402


def use(eng, mode):
    if mode == "scan":
        img, n, end = coracle.gen_log(64 << 20, 5, ksize=64, vsize=256)
        eng.scan_dev(torch.from_numpy(img).to("cuda:0"))
    elif mode == "host":
        img, n, end = coracle.gen_log(8 << 20, 5, ksize=64, vsize=256)
        eng.scan_host(img)
    elif mode == "merge":
        files, kw = MC.small_cases()["gen1"]
        d = [(torch.from_numpy(np.ascontiguousarray(f[0])).to("cuda:0"), f[1], f[2]) for f in files]
        eng.merge_dev(d, kw["active_fid"], kw["active_off"], kw["max_file_size"], kw["now"])
    elif mode == "bigscan":   # multi-GiB workspace, as the parity module's 4.5 GiB case
        img, n, end = coracle.gen_log(9 << 29, 10, ksize=64, vsize=256)
        res, tup = eng.scan_dev(torch.from_numpy(img).to("cuda:0"))
        assert res.n_entries == n
    elif mode == "crcmerge":   # a merge that stops at a file with a bad CRC
        files, kw = MC.small_cases()["crc_corrupt"]
        d = [(torch.from_numpy(np.ascontiguousarray(f[0])).to("cuda:0"), f[1], f[2]) for f in files]
        out = eng.merge_dev(d, kw["active_fid"], kw["active_off"], kw["max_file_size"], kw["now"])
        assert out["result"].bad_file == 1
    elif mode == "encode":
        files, kw = MC.small_cases()["gen1"]
        d = [(torch.from_numpy(np.ascontiguousarray(f[0])).to("cuda:0"), f[1], False) for f in files]
        eng.merge_dev(d, 0, 0, 1 << 40, 0)


def main():
    modes = sys.argv[1:] or ["scan", "host", "merge"]
    for mode in modes:
        for cycle in range(4):
            eng = Engine(0)
            use(eng, mode)
            torch.cuda.synchronize()
            eng.close()
            for n in (1 << 10, 1 << 16, 3 << 20):
                a = (np.arange(n) % 251).astype(np.uint8)
                assert np.array_equal(torch.from_numpy(a).to("cuda:0").cpu().numpy(), a)
            torch.cuda.synchronize()
            print(f"{mode} cycle {cycle} ok {time.time():.0f}", flush=True)


if __name__ == "__main__":
    main()
