"""Scan throughput on adversarial logs (the serial fallbacks' speed was unmeasured).

Each case is a block of whole entries from the golden-fixture generators (tests/golden/make_golden.py),
cut at the oracle's end_off and tiled to --mib MiB, so the log is one valid chain of entries:
  embedded  values holding complete valid entries and zero runs (speculative resyncs land inside values)
  binary    random binary keys/values (random bytes that decode as plausible headers)
  mixed     every header field varied, keys/values 0..300 B
  txlog     Tx.Commit entries: snowflake TxIDs (10-byte varints), TxStat 1, 1-16 entries per tx
  tiny      1-byte keys, empty values (11-B entries: the densest regions)
  big       64 KiB-scale values (regions fully inside one value)
Every case is checked against the C oracle (status, end_off, n_entries, tuples) before it is timed.
Prints one JSON line per case. Usage: python tools/adversarial.py [--mib 256] [--reps 5] [--cases a,b]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

from oracle import coracle  # noqa: E402  checker only
import make_golden as MG  # noqa: E402


def block(case: str) -> np.ndarray:
    if case == "embedded":
        raw = MG.embedded(21, 1 << 20)
    elif case == "binary":
        raw = MG.binary_values(22, 1 << 20)
    elif case == "mixed":
        raw = MG.mixed(23, 1 << 20)
    elif case == "big":
        raw = MG.big_values(24, 4 << 20)
    elif case == "txlog":   # Tx.Commit writes (tx.go:156-206): snowflake TxIDs (10-byte varints), TxStat 1
        import random
        rng = random.Random(25)
        parts, used, ms = [], 0, 1_700_000_000_000
        while used < (1 << 20):
            ms += rng.randrange(1, 50)
            tx = (ms << 22) | (rng.randrange(1023) << 12) | rng.randrange(4096)
            for _ in range(rng.randrange(1, 17)):
                e = MG.ent(key=MG.alpha(rng, rng.randrange(16, 65)), value=MG.alpha(rng, rng.randrange(32, 513)),
                           tx_id=tx, tx_stat=1, expired_at=rng.choice([0] * 9 + [1_700_000_000 + rng.randrange(10**6)]))
                parts.append(e)
                used += len(e)
        raw = b"".join(parts)
    elif case == "tiny":
        e = MG.ent(key=b"k", value=b"")
        raw = e * ((1 << 20) // len(e))
    else:
        raise ValueError(case)
    img = np.frombuffer(raw, dtype=np.uint8)
    r, _ = coracle.scan(img)
    return img[: r.end_off].copy()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--cases", default="embedded,binary,mixed,txlog,tiny,big")
    args = ap.parse_args()
    import torch
    from lazydb_amd import Engine
    eng = Engine(0)
    for case in args.cases.split(","):
        b = block(case)
        n_rep = max(1, (args.mib << 20) // len(b))
        img = np.concatenate([np.tile(b, n_rep), np.zeros(64, np.uint8)])
        ref, rt = coracle.scan(img)
        d = torch.from_numpy(img).to("cuda:0")
        cap = img.size // 10 + 16
        out = eng.alloc_out(cap)
        res = eng.alloc_result()
        eng.scan_dev_async(d, out=out, cap=cap, result=res)
        torch.cuda.synchronize()
        r, tup = eng.scan_dev(d, cap=cap)
        ok = (r.status, r.end_off, r.n_entries) == (ref.status, ref.end_off, ref.n_entries) and \
            np.array_equal(tup["pos"], rt["pos"]) and np.array_equal(tup["k_size"], rt["k_size"]) and \
            np.array_equal(tup["v_size"], rt["v_size"])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            eng.scan_dev_async(d, out=out, cap=cap, result=res)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.reps
        eng.timing_split(1)   # a second pass with events between the stages, for the split only
        for _ in range(args.reps):
            eng.scan_dev_async(d, out=out, cap=cap, result=res)
        torch.cuda.synchronize()
        ph = eng.timing_tail()
        sw = eng.timing_sweep()[0]
        u, a, p, nl = eng.timing_split(0)
        print(json.dumps({"case": case, "bytes": int(ref.end_off), "entries": int(ref.n_entries),
                          "avg_entry_B": round(ref.end_off / max(1, ref.n_entries), 1), "verified": bool(ok),
                          "ms": round(ms, 3), "GiB_per_s": round(ref.end_off / (ms * 1e-3) / 2**30, 1),
                          "n_regions": int(r.n_regions), "n_fast": int(r.n_fast), "n_repairs": int(r.n_repairs),
                          "n_broken_after_walk": int(r.n_broken), "k_uniform_ms": round(u, 4), "k_sweep_ms": round(sw, 4), "k_region_ms": round(a, 4), "pipeline_ms": round(p, 4),
                          "n_sweep": int(r.n_sweep), "tail_phases_ms": [round(x, 4) for x in ph]}),
              flush=True)
        del d, out, res
        torch.cuda.empty_cache()
    eng.close()


if __name__ == "__main__":
    main()
