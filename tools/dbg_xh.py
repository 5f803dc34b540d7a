"""Debug helper: the hash-partitioned merge on small cases at several simulated rank counts."""
import sys
sys.path.insert(0, "/root/repo")
import numpy as np, torch
from lazydb_amd import Engine, xmerge as X, _native as N
from tests import merge_cases as MC
engs = [Engine(0) for _ in range(4)]
for name in ("gen1", "gen2"):
    files, kw = MC.small_cases()[name]
    d = [(torch.from_numpy(np.ascontiguousarray(f[0])).to("cuda:0"), f[1], f[2]) for f in files]
    for world in (2, 3):
        blocks = [[d[i] for i in b] for b in np.array_split(np.arange(len(d)), world)]
        print(name, world, [[f[1] for f in b] for b in blocks], "active", kw["active_fid"], flush=True)
        routes = [X.route_phase(engs[r], blocks[r], world) for r in range(world)]
        print("  n_records", [int(ro["result"].n_records) for ro in routes], "counts", [list(ro["counts"]) for ro in routes])
        for r in range(world):
            lr = torch.ones(max(int(routes[r]["result"].n_records), 1), dtype=torch.uint8, device="cuda:0")
            out = engs[r].merge_dev(blocks[r], kw["active_fid"], kw["active_off"], kw["max_file_size"], kw["now"],
                                    fetch_pos=False, last=lr)
            print("  apply", r, "rc", out["rc"], "status", out["result"].status, "bad", out["result"].bad_file, flush=True)
