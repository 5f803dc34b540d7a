"""Scan one synthetic image a few times on cuda:0 (for rocprofv3 kernel traces of a single workload).
usage: python tools/scan_one.py <cfg: 1|2|3|4|w|adv:<case>> [reps] [io]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from lazydb_amd import Engine
    cfg = sys.argv[1] if len(sys.argv) > 1 else "w"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    io_arg = int(sys.argv[3]) if len(sys.argv) > 3 else None
    sys.argv = sys.argv[:1]
    import bench
    img, n, end, wl, io = bench.make_image(cfg if cfg == "w" else int(cfg), 0)
    io = io_arg if io_arg is not None else (io or 0)
    eng = Engine(0)
    d = torch.from_numpy(img).to("cuda:0")
    eng.reserve(img.size)
    res, _ = eng.scan_dev(d, io_type=io, cap=n + 1024)
    out, rb = eng.alloc_out(n + 1024, 0), eng.alloc_result()
    bench.settle(lambda: eng.scan_dev_async(d, io_type=io, out=out, cap=n + 1024, result=rb), 150.0)   # clocks (DVFS)
    torch.cuda.synchronize()
    eng.timing_split(1)
    t0 = time.perf_counter()
    for _ in range(reps):
        res, _ = eng.scan_dev(d, io_type=io, cap=n + 1024)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ph = eng.timing_tail()
    sw = eng.timing_sweep()[0]
    u, m, tot, k = eng.timing_split(0)
    print(f"{wl}: status {res.status} entries {res.n_entries} end {res.end_off} run {res.n_run} sweep {res.n_sweep} "
          f"fast {res.n_fast}/{res.n_regions} repairs {res.n_repairs} broken {res.n_broken} | {dt * 1e3:.3f} ms/scan wall, "
          f"k_uniform {u:.4f} k_sweep {sw:.4f} k_region {m:.4f} pipeline {tot:.4f} ms; phases " + " ".join(f"{x:.4f}" for x in ph))
    eng.close()


if __name__ == "__main__":
    main()
