"""Generate the golden fixtures in tests/golden/ (committed; re-run to regenerate).

Each fixture is an input log image `<name>.bin` plus its expected replay result
in `golden.json`: the status and end offset at which (*LogFile).ReadLogEntry
stops the index.go loop, and the tuples (offset, hdr_size, enc_hdr_size, stat,
k_size, v_size) in file order.  Expected results come from the pure-Python
restatement (oracle/pyoracle.py) and are cross-checked against the C
restatement (oracle/ldb_oracle.c) before being written.

The reference (Go) cannot run here, so these are self-generated vectors whose
codec is pinned by the reference's own literal vectors
(logfile/log_entry_test.go, db_test.go) in tests/test_oracle_golden.py.
"""
from __future__ import annotations

import json
import os
import random
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))

from oracle import coracle  # noqa: E402
from oracle import pyoracle as P  # noqa: E402

ALPHA = b"0123456789abcdefghijklmnopqrstuvwxyz"


def alpha(rng: random.Random, n: int) -> bytes:
    return bytes(rng.choice(ALPHA) for _ in range(n))


def ent(**kw) -> bytes:
    return P.encode_entry(P.Entry(**kw))


def image(parts: list[bytes], size: int) -> bytes:
    b = b"".join(parts)
    assert len(b) <= size, (len(b), size)
    return b + bytes(size - len(b))


def ref_read_entries() -> bytes:
    # logfile/log_file_test.go:42-51
    es = [
        ent(expired_at=123332, stat=2),
        ent(expired_at=123332, stat=1),
        ent(expired_at=994332343, stat=2),
        ent(expired_at=7844332343, key=b"k1"),
        ent(expired_at=99400542343, value=b"test test"),
        ent(expired_at=8847333912, key=b"k2", value=b"test"),
        ent(expired_at=8847333912, stat=1, key=b"k3", value=b"some data"),
        ent(expired_at=8847333912, stat=1, tx_id=100, tx_stat=1, key=b"k3", value=b"some data"),
    ]
    return image(es, 4096)


def ref_rollover() -> bytes:
    # db_test.go:183-239: 32-B key + 32-B value = 74-B entries, MaxLogFileSize=150 -> 2 per file
    rng = random.Random(7)
    es = [ent(key=b"kvstore-bench-key------%09d" % i, value=alpha(rng, 32)) for i in (1, 2)]
    assert all(len(e) == 74 for e in es)
    return image(es, 150)


def mixed(seed: int, size: int, maxv: int = 300) -> bytes:
    rng = random.Random(seed)
    parts, used = [], 0
    while True:
        kl = rng.choice([0, 0, 1, 2, 7, 16, 64, rng.randrange(0, 200)])
        vl = rng.choice([0, 0, 1, 3, 31, 256, rng.randrange(0, maxv)])
        e = ent(stat=rng.choice([0, 0, 0, 1, 2]),
                expired_at=rng.choice([0, 0, 1676969769, rng.randrange(-(1 << 62), 1 << 62)]),
                tx_id=rng.choice([0, 0, 11111111, rng.randrange(0, 1 << 64)]),
                tx_stat=rng.choice([0, 0, 1, 2]),
                key=alpha(rng, kl), value=alpha(rng, vl))
        if used + len(e) > size - 64:
            break
        parts.append(e)
        used += len(e)
    return image(parts, size)


def binary_values(seed: int, size: int) -> bytes:
    """Random binary values (stress for the speculative resync heuristic)."""
    rng = random.Random(seed)
    parts, used = [], 0
    while True:
        e = ent(key=rng.randbytes(rng.randrange(1, 40)), value=rng.randbytes(rng.randrange(0, 600)))
        if used + len(e) > size - 64:
            break
        parts.append(e)
        used += len(e)
    return image(parts, size)


def embedded(seed: int, size: int) -> bytes:
    """Values that contain complete, valid encoded entries (and zero runs): a speculative
    parallel walk that resyncs inside a value must be repaired."""
    rng = random.Random(seed)
    parts, used = [], 0
    while True:
        inner = b"".join(ent(key=alpha(rng, rng.randrange(1, 20)), value=alpha(rng, rng.randrange(0, 120)))
                         for _ in range(rng.randrange(1, 12)))
        pad = bytes(rng.randrange(0, 50))
        e = ent(key=alpha(rng, 8), value=pad + inner + pad + alpha(rng, rng.randrange(0, 30)))
        if used + len(e) > size - 64:
            break
        parts.append(e)
        used += len(e)
    return image(parts, size)


def big_values(seed: int, size: int) -> bytes:
    rng = random.Random(seed)
    parts, used = [], 0
    while True:
        vl = rng.choice([16, 100, 5000, 5121, 10239, 20000, rng.randrange(0, 30000)])
        e = ent(key=alpha(rng, 64), value=alpha(rng, vl))
        if used + len(e) > size:
            break
        parts.append(e)
        used += len(e)
    return image(parts, size)


def with_tail_window(size: int) -> bytes:
    """Last entry fits in the file but its 38-byte header window does not (Appendix B.1)."""
    rng = random.Random(3)
    body = mixed(11, size - 200)[: size - 200]
    st, end, _ = P.scan(body)
    body = body[:end]
    small = ent(key=b"k", value=b"v")  # 12 bytes < 38
    filler = ent(key=alpha(rng, 10), value=alpha(rng, size - len(body) - len(small) - 16))
    img = body + filler + small
    return image([img], len(img))


def exact_end(size: int) -> bytes:
    """Last entry ends exactly at the bound: accepted under FileIO, dropped under Mmap."""
    rng = random.Random(5)
    parts, used = [], 0
    while used < size - 400:
        e = ent(key=alpha(rng, 20), value=alpha(rng, 100))
        parts.append(e)
        used += len(e)
    last = size - used
    hdr = len(ent(key=alpha(rng, 20), value=b"x" * 200)) - 220
    parts.append(ent(key=alpha(rng, 20), value=alpha(rng, last - hdr - 20)))
    b = b"".join(parts)
    assert len(b) == size, (len(b), size)
    return b


def corrupt(src: bytes, at_entry: int) -> bytes:
    st, end, tup = P.scan(src)
    off, h, eh, stat, k, v = tup[at_entry]
    b = bytearray(src)
    idx = off + h + k + v - 1 if (k + v) else off + 4  # last key/value byte, else the stat byte
    b[idx] ^= 0x5A
    return bytes(b)


def kv_eof() -> bytes:
    """A header whose k+v runs past the end of the file."""
    rng = random.Random(9)
    parts = [ent(key=alpha(rng, 10), value=alpha(rng, 50)) for _ in range(20)]
    b = b"".join(parts)
    tail = ent(key=alpha(rng, 10), value=alpha(rng, 500))
    return b + tail[:200]


def sentinel_mid() -> bytes:
    rng = random.Random(13)
    a = b"".join(ent(key=alpha(rng, 10), value=alpha(rng, 90)) for _ in range(40))
    c = b"".join(ent(key=alpha(rng, 10), value=alpha(rng, 90)) for _ in range(40))
    return a + bytes(64) + c + bytes(100)


def zero_len_entries() -> bytes:
    rng = random.Random(17)
    parts = []
    for i in range(300):
        parts.append(ent(tx_id=i + 1))  # key == value == "" but crc != 0: a valid entry
        if i % 7 == 0:
            parts.append(ent(key=alpha(rng, 3), value=b""))
    return image(parts, 8192)


def noncanonical() -> bytes:
    """Headers with padded (non-minimal) varints: hdr_size != enc_hdr_size, and stat/txstat > 2."""
    rng = random.Random(21)
    out = []
    for i in range(200):
        key, val = alpha(rng, rng.randrange(1, 30)), alpha(rng, rng.randrange(0, 200))
        fields = [rng.randrange(0, 1 << 40), rng.randrange(0, 1 << 20), rng.randrange(0, 5), len(key), len(val)]
        hdr = bytearray([rng.choice([0, 1, 2, 3, 200])])
        for f in fields:
            enc = bytearray(P.put_varint(f))
            for _ in range(rng.randrange(0, 3)):  # pad with continuation bytes
                if len(enc) < 9:
                    enc[-1] |= 0x80
                    enc.append(0)
            hdr += enc
        body = bytes(hdr) + key + val
        if len(body) + 4 > 38 + len(key) + len(val):
            continue
        crc = __import__("zlib").crc32(body)
        out.append(struct.pack("<I", crc) + body)
    return image(out, sum(map(len, out)) + 64)


def noncanonical5() -> bytes:
    """5-byte padded expiredAt / txID varints (re-encoded shorter by EncodeEntry) among normal entries."""
    rng = random.Random(23)
    out = []
    for i in range(300):
        key, val = alpha(rng, rng.randrange(1, 20)), alpha(rng, rng.randrange(0, 100))
        if i % 3:
            out.append(ent(key=key, value=val, expired_at=rng.choice([0, 5, 1676969769])))
            continue
        fields = [rng.choice([0, 1, 63, 1000]), rng.choice([0, 7]), 0, len(key), len(val)]
        hdr = bytearray([0])
        for j, f in enumerate(fields):
            enc = bytearray(P.put_varint(f))
            if j == i % 2 or rng.random() < 0.3:
                while len(enc) < 5:
                    enc[-1] |= 0x80
                    enc.append(0)
            hdr += enc
        body = bytes(hdr) + key + val
        out.append(struct.pack("<I", __import__("zlib").crc32(body)) + body)
    return image(out, sum(map(len, out)) + 64)


def malformed(seed: int) -> list[tuple[str, bytes]]:
    """Random header windows after a valid prefix; keep one image per ReadLogEntry outcome,
    plus an accepted entry whose decoded header size is <= 4 (getEntryCrc returns 0)."""
    rng = random.Random(seed)
    prefix = b"".join(ent(key=alpha(rng, 5), value=alpha(rng, 40)) for _ in range(30))
    names = {P.ERR_MALFORMED: "malformed_panic", P.ERR_CRC: "malformed_crc", P.EOF_SENTINEL: "malformed_sentinel",
             P.EOF_KV: "malformed_kv_eof"}
    found: dict[int, bytes] = {}
    weird_ok = None
    for _ in range(60000):
        w = bytearray(rng.randbytes(38))
        if rng.random() < 0.5:
            for j in range(5, 38):
                if rng.random() < 0.6:
                    w[j] |= 0x80
        if rng.random() < 0.3:
            w[0:4] = b"\0\0\0\0"
        img = prefix + bytes(w) + alpha(rng, 300)
        st, e, es, h = P.read_log_entry(img, 0, len(prefix))
        if st in names and st not in found:
            found[st] = img
        if weird_ok is None and st == P.OK and h <= 4:
            weird_ok = img
        if len(found) == len(names) and weird_ok is not None:
            break
    out = [(names[k], v) for k, v in sorted(found.items())]
    if weird_ok is not None:
        out.append(("weird_small_header", weird_ok))
    return out


def fixtures() -> list[tuple[str, bytes, list[int]]]:
    fx = [
        ("ref_read_entries", ref_read_entries(), [0, 1]),
        ("ref_rollover", ref_rollover(), [0, 1]),
        ("mixed_64k", mixed(1, 65536), [0, 1]),
        ("mixed_200k", mixed(2, 200000, 1000), [0]),
        ("binary_values", binary_values(3, 131072), [0]),
        ("embedded_entries", embedded(4, 131072), [0, 1]),
        ("big_values", big_values(5, 262144), [0, 1]),
        ("tail_window", with_tail_window(20000), [0, 1]),
        ("exact_end", exact_end(30000), [0, 1]),
        ("kv_eof", kv_eof(), [0, 1]),
        ("sentinel_mid", sentinel_mid(), [0]),
        ("zero_len_entries", zero_len_entries(), [0]),
        ("noncanonical", noncanonical(), [0]),
        ("noncanonical5", noncanonical5(), [0, 1]),
        ("all_zero", bytes(10000), [0, 1]),
        ("tiny_37", ent(key=b"k", value=b"v") + bytes(25), [0, 1]),
        ("empty", b"", [0, 1]),
    ]
    m = mixed(6, 60000)
    fx.append(("crc_corrupt", corrupt(m, 40), [0]))
    fx.append(("crc_corrupt_first", corrupt(m, 0), [0]))
    for name, img in malformed(8):
        fx.append((name, img, [0, 1]))
    return fx


def main():
    meta = []
    total = 0
    for name, img, ios in fixtures():
        with open(os.path.join(HERE, name + ".bin"), "wb") as f:
            f.write(img)
        total += len(img)
        for io in ios:
            st, end, tup = P.scan(img, io)
            arr = np.frombuffer(img, dtype=np.uint8)
            res, ct = coracle.scan(arr, io)
            assert res.status == st and res.end_off == end and res.n_entries == len(tup), (name, io, st, res.status)
            if tup:
                pos = [P.pack_pos(o, h, eh, s) for (o, h, eh, s, k, v) in tup]
                assert list(ct["pos"]) == pos and list(ct["k_size"]) == [t[4] for t in tup], name
            meta.append({"name": name, "io_type": io, "len": len(img), "status": st, "end_off": end,
                         "tuples": [list(t) for t in tup]})
            print(f"{name:24s} io={io} len={len(img):7d} status={st:2d} end={end:7d} n={len(tup)}")
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, separators=(",", ":"))
    print("total bytes", total)


if __name__ == "__main__":
    main()
