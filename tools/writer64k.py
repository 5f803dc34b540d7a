"""The writer mix with binary values up to 64 KiB (test_gpu_sweep.py's, scaled): coverage of the sweep tier
and the scan time on cuda:0. usage: python tools/writer64k.py [MiB]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from lazydb_amd import Engine
    from oracle import coracle
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    w, nw, _ = coracle.gen_writer_log(mib << 20, 17, vmax=65536)
    ref, rt = coracle.scan(w)
    eng = Engine(0)
    d = torch.from_numpy(w).to("cuda:0")
    res, tup = eng.scan_dev(d, cap=nw + 1024)
    ok = (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries) and tup.tobytes() == rt.tobytes()
    out, rb = eng.alloc_out(nw + 1024, 0), eng.alloc_result()
    for _ in range(5):
        eng.scan_dev_async(d, out=out, cap=nw + 1024, result=rb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        eng.scan_dev_async(d, out=out, cap=nw + 1024, result=rb)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 20 * 1e3
    print(f"writer 64K {mib} MiB: entries {nw} verified {ok} n_sweep {res.n_sweep} regions {res.n_regions} "
          f"{ms:.3f} ms/scan wall, {w.size / ms / 1e6:.1f} GB/s")
    assert ok


if __name__ == "__main__":
    main()
