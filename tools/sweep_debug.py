"""Where and why the sweep tier ended on a log (diagnostics): runs the scan on cuda:0, reads the run records
and the control block (ldb_debug_sweep_state), and prints the runs around the tier's end beside the
oracle's chain. usage: python tools/sweep_debug.py [writer|zipf|adv:<case>] [mib] [seed]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SWRUN = np.dtype([("E", "<u8"), ("X", "<u8"), ("n", "<u8"), ("flags", "<u4"), ("ncand", "<u4"), ("lo", "<u8"),
                  ("hi", "<u8"), ("base", "<u8"), ("pad", "<u8")])
SWCTL = np.dtype([("xs", "<u8"), ("ks", "<u8"), ("xe", "<u8"), ("ke", "<u8"), ("ncov", "<u8"), ("fail", "<u8"),
                  ("stop", "<u8"), ("done0", "<u8"), ("done1", "<u8"), ("state", "<u8"), ("nrun", "<u8"),
                  ("pad", "<u8", (5,))])


def main():
    import torch
    from lazydb_amd import Engine
    from lazydb_amd import _native as N
    from oracle import coracle
    kind = sys.argv[1] if len(sys.argv) > 1 else "writer"
    mib = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    seed = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    if kind == "writer":
        img, n, _ = coracle.gen_writer_log(mib << 20, seed)
    elif kind.startswith("adv:"):   # a tools/adversarial.py case tiled to mib MiB
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import adversarial
        b = adversarial.block(kind[4:])
        img = np.concatenate([np.tile(b, max(1, (mib << 20) // len(b))), np.zeros(64, np.uint8)])
        n = int(coracle.scan(img)[0].n_entries)
    else:
        img, n, _ = coracle.gen_log(mib << 20, seed, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
    ref, rt = coracle.scan(img, tuple_kind=1)
    eng = Engine(0)
    d = torch.from_numpy(img).to("cuda:0")
    res, _ = eng.scan_dev(d, cap=n + 1024)
    torch.cuda.synchronize()
    L = N.lib()
    L.ldb_debug_sweep_state.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
    runs = np.zeros(4096, dtype=SWRUN)
    ctl = np.zeros(1, dtype=SWCTL)
    N.check(L.ldb_debug_sweep_state(eng.ctx, img.size, runs.ctypes.data, 4096, ctl.ctypes.data), "debug state")
    c = ctl[0]
    print(f"n {res.n_entries}/{ref.n_entries} n_run {res.n_run} n_sweep {res.n_sweep} status {res.status}")
    print({k: int(c[k]) for k in ("xs", "ks", "xe", "ke", "ncov", "fail", "stop", "nrun")})
    nrun = int(c["nrun"])
    xe = int(c["xe"])
    offs = rt["offset"].astype(np.int64)
    r_end = next((r for r in range(nrun) if int(runs[r]["lo"]) <= xe < int(runs[r]["hi"]) or int(runs[r]["hi"]) > xe), nrun - 1)
    for r in range(max(0, r_end - 2), min(nrun, r_end + 3)):
        q = runs[r]
        lo, hi = int(q["lo"]), int(q["hi"])
        true_first = offs[(offs >= lo) & (offs < hi)]
        print(f"run {r}: [{lo}, {hi}) E {int(q['E']) if q['E'] != 2**64 - 1 else -1} X {int(q['X'])} n {int(q['n'])} "
              f"flags {int(q['flags']) & 0xFF:#x} tag {int(q['flags']) >> 8} ncand {int(q['ncand'])} base {int(q['base'])} | "
              f"true first start {int(true_first[0]) if true_first.size else -1}, true starts {true_first.size}")
    eng.close()


if __name__ == "__main__":
    main()
