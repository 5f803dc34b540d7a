"""The sweep tier on cuda:0 against the C oracle: Zipf logs (config 3's shape, smaller), long values, corrupt
bytes at span edges, writer mix, both IO rules and tuple kinds. Prints the tier's share (n_sweep) and times.
usage: python tools/sweep_check.py [mib]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from lazydb_amd import Engine
    from oracle import coracle
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    big = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    eng = Engine(0)
    cases = []
    img, n, end = coracle.gen_log(mib << 20, 3, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
    cases.append(("zipf4096", img, n))
    img2, n2, _ = coracle.gen_log(mib << 20, 4, ksize=64, value_mode=1, zipf_s=1.05, zipf_max=16384)
    cases.append(("zipf16384", img2, n2))
    w, nw, _ = coracle.gen_writer_log(min(mib, 32) << 20, 5)
    cases.append(("writer", w, nw))
    # corruptions in the Zipf log: the first and last byte of an entry's CRC span, a byte at a window edge
    _, rt = coracle.scan(img)
    pos = rt["pos"] & ((1 << 40) - 1)
    hs = (rt["pos"] >> 40) & 63
    sz = hs + rt["k_size"].astype(np.int64) + rt["v_size"].astype(np.int64)
    rng = np.random.default_rng(7)
    for tag, f in (("first", lambda i: int(pos[i]) + 4), ("last", lambda i: int(pos[i] + sz[i]) - 1),
                   ("win", lambda i: (int(pos[i]) + int(sz[i]) // 2) | 255)):
        i = int(rng.integers(len(pos) // 4, len(pos) - 2))
        c = img.copy()
        c[f(i)] ^= 0x40
        cases.append((f"corrupt_{tag}", c, n))
    if big:
        zb, nb, _ = coracle.gen_log(big << 20, 11, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
        cases.append((f"zipf_{big}MiB", zb, nb))
    bad = 0
    for name, im, n0 in cases:
        d = torch.from_numpy(im).to("cuda:0")
        for io in (0, 1):
            for kind in (0, 1):
                res, tup = eng.scan_dev(d, io_type=io, kind=kind, cap=n0 + 1024)
                ref, rt2 = coracle.scan(im, io_type=io, tuple_kind=kind)
                ok = (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries)
                m = min(res.n_entries, n0 + 1024)
                if ok:
                    for k in rt2.dtype.names:
                        if not np.array_equal(tup[k][:m], rt2[k][:m]):
                            ok = False
                            print("  field mismatch", k, np.nonzero(tup[k][:m] != rt2[k][:m])[0][:5])
                            break
                bad += 0 if ok else 1
                print(f"{name:16s} io {io} kind {kind}: {'OK ' if ok else 'BAD'} status {res.status}/{ref.status} "
                      f"n {res.n_entries}/{ref.n_entries} end {res.end_off}/{ref.end_off} run {res.n_run} sweep "
                      f"{res.n_sweep} regions {res.n_regions} fast {res.n_fast}", flush=True)
        eng.timing_split(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            res, _ = eng.scan_dev(d, cap=n0 + 1024)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 10
        sw, fin = eng.timing_sweep()
        u, mm, tot, k = eng.timing_split(0)
        print(f"   {name}: {dt * 1e3:.3f} ms/scan wall, k_uniform {u:.4f} k_sweep {sw:.4f} fin {fin:.4f} k_scan_main {mm:.4f} "
              f"pipeline {tot:.4f} ms = {im.size / tot / 1e6:.1f} GB/s", flush=True)
    eng.close()
    print("ALL OK" if bad == 0 else f"{bad} BAD")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
