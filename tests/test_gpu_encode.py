"""GPU parity of the batch writeLogEntry (ldb_encode_entries_dev) against EncodeEntry restated twice
(oracle/pyoracle.py zlib and oracle/ldb_oracle.c, both pinned to logfile/log_entry_test.go:18-32) and
the rollover loop of db.go:473-523 (pinned to db_test.go:182-229)."""
import random

import numpy as np
import pytest

from oracle import coracle
from oracle import pyoracle as P

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(gpu_engine):
    return gpu_engine


def build(entries):
    from lazydb_amd import _native as N
    blob = bytearray()
    items = np.zeros(len(entries), dtype=N.ENCODE_ITEM)
    for i, e in enumerate(entries):
        items[i]["key_off"] = len(blob)
        blob += e.key
        items[i]["value_off"] = len(blob)
        blob += e.value
        items[i]["k_size"] = len(e.key)
        items[i]["v_size"] = len(e.value)
        items[i]["expired_at"] = e.expired_at
        items[i]["tx_id"] = e.tx_id
        items[i]["tx_stat"] = e.tx_stat
        items[i]["stat"] = e.stat
    return items, bytes(blob)


def check(eng, entries, active_fid, active_off, max_size):
    import torch
    items, blob = build(entries)
    d_blob = torch.frombuffer(bytearray(blob) + bytearray(16), dtype=torch.uint8).to("cuda:0")
    out = eng.encode_entries(items, d_blob, active_fid, active_off, max_size)
    stream, pos, segs, efid, eoff = P.write_entries(entries, active_fid, active_off, max_size)
    r = out["result"]
    assert out["stream"].cpu().numpy().tobytes() == stream
    assert [(int(p["fid"]), int(p["offset"]), int(p["entry_size"])) for p in out["pos"]] == pos
    assert [(int(s["fid"]), int(s["file_off"]), int(s["stream_off"]), int(s["n_bytes"])) for s in out["segments"]] \
        == segs
    assert (r.end_fid, r.end_off, r.n_emit, r.emit_bytes) == (efid, eoff, len(entries), len(stream))
    # C restatement agrees byte for byte on every entry
    o = 0
    for e in entries:
        c = coracle.encode_entry(e.stat, e.expired_at, e.tx_id, e.tx_stat, e.key, e.value)
        assert stream[o:o + len(c)] == c
        o += len(c)


def test_reference_vectors_and_rollover(eng):
    # logfile/log_entry_test.go:18-32 entries, then db_test.go:182-229 (74-B entries, MaxLogFileSize 150)
    ents = [P.Entry(), P.Entry(expired_at=1676969769, stat=2, tx_id=11111111, tx_stat=2, key=b"a", value=b"abc"),
            P.Entry(stat=1)]
    items, blob = build(ents)
    check(eng, ents, 0, 0, 1 << 20)
    key = lambda n: b"kvstore-bench-key------" + b"%09d" % n
    ents = [P.Entry(key=key(i), value=bytes(range(65, 97))) for i in (1, 2, 3)]
    check(eng, ents, 1, 0, 150)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_batches(eng, seed):
    rng = random.Random(seed)
    ents = []
    for _ in range(rng.choice([1, 17, 3000, 20000])):
        ents.append(P.Entry(stat=rng.choice([0, 0, 1, 2]),
                            expired_at=rng.choice([0, 0, -1, 1 << 40, -(1 << 62), 1676969769]),
                            tx_id=rng.choice([0, 1, 11111111, (1 << 64) - 1, 1 << 63]),
                            tx_stat=rng.choice([0, 1, 2, 65535]),
                            key=bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 1, 16, 64]))),
                            value=bytes(rng.getrandbits(8) for _ in range(rng.choice([0, 3, 256, 5000])))))
    check(eng, ents, 7, rng.choice([0, 100, 4000]), rng.choice([1 << 12, 1 << 16, 1 << 30]))
