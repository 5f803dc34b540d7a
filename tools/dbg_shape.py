"""Debug: run test_run_prefix_shapes' variants for one shape and print the first tuple mismatch."""
import os, random, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch
from lazydb_amd import Engine
from oracle import coracle
from test_gpu_parity import _fixed_log

eng = Engine(0)
klen, vlen, exp, txid = [int(a) for a in sys.argv[1:5]]
rng = random.Random(klen * 7 + vlen)
n = 3000 if vlen < 1000 else 600
run = _fixed_log(n, klen, vlen, rng.randrange(1 << 30), expired_at=exp, tx_id=txid)
esz = len(run) // n
other = coracle.gen_log(200_000, 6, ksize=16, vsize=40)
bad = 0
for ti, tail in enumerate((b"", bytes(37), bytes(9000), bytes(other[0][: other[2]]) + bytes(300))):
    base = np.frombuffer(run + tail, np.uint8).copy()
    variants = [base, base[: (n // 2) * esz + 3].copy(), base[: (n - 1) * esz + 30].copy()]
    for k in (0, 1, n // 4, n - 1):
        im = base.copy()
        im[k * esz + rng.choice([0, 5, esz - 1])] ^= 0x40
        variants.append(im)
    for vi, im in enumerate(variants):
        d = torch.from_numpy(im).cuda()
        for io in (0, 1):
            res, tup = eng.scan_dev(d, io_type=io, kind=0)
            ref, rt = coracle.scan(im, io, tuple_kind=0)
            same = (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries)
            pe = np.nonzero(tup["pos"] != rt["pos"])[0] if same else np.array([-1])
            if not same or pe.size:
                bad += 1
                i = int(pe[0]) if pe.size else -1
                print(f"tail {ti} var {vi} io {io}: res {res.as_dict()} ref {(ref.status, ref.end_off, ref.n_entries)} "
                      f"esz {esz} nbad {pe.size} first {i} got {int(tup['pos'][i]) & ((1<<40)-1) if i >= 0 else None:} "
                      f"want {int(rt['pos'][i]) & ((1<<40)-1) if i >= 0 else None} got_hi {int(tup['pos'][i]) >> 40 if i >= 0 else None} "
                      f"want_hi {int(rt['pos'][i]) >> 40 if i >= 0 else None} last {pe[-5:] if pe.size else None}")
print("bad", bad)
