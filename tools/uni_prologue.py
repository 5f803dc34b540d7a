"""k_uniform's fixed cost (workgroup setup: LP2 block, combine tables, memo, header probes) from scans
of small equal-entry images, where the verify loop itself is a few microseconds.
usage: python tools/uni_prologue.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from lazydb_amd import Engine
    from oracle import coracle
    eng = Engine(0)
    for mib in (1, 16, 64, 256):
        img, n, end = coracle.gen_log(mib << 20, 1, ksize=64, vsize=256)
        d = torch.from_numpy(img).to("cuda:0")
        for _ in range(3):
            eng.scan_dev(d, cap=n + 16)
        torch.cuda.synchronize()
        eng.timing_split(1)
        for _ in range(20):
            eng.scan_dev(d, cap=n + 16)
        torch.cuda.synchronize()
        u, m, tot, k = eng.timing_split(0)
        print(f"{mib:4d} MiB: k_uniform {u * 1e3:8.1f} us  pipeline {tot * 1e3:8.1f} us  "
              f"({(end / (u * 1e-3)) / 1e12:.2f} TB/s incl. setup)", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
