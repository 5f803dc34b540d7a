"""Merge/GC test cases shared by the CPU oracle tests and the GPU parity tests.

Each case is (files, kwargs): files = [(uint8 ndarray image, fid, is_target)] in ascending fid,
kwargs = active_fid / active_off / max_file_size / now / io_type for Merge (db.go:383-427).
Images come from the oracle's generators (writeLogEntry format) and the committed golden fixtures.
"""
from __future__ import annotations

import os

import numpy as np

from oracle import coracle

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NOW = 1_700_000_000


def ref_key(n: int) -> bytes:   # db_test.go:336-338 GetKey
    return b"kvstore-bench-key------" + b"%09d" % n


def _log(entries, size: int | None = None) -> np.ndarray:
    buf = b"".join(coracle.encode_entry(**e) for e in entries)
    img = np.zeros(len(buf) if size is None else size, dtype=np.uint8)
    img[: len(buf)] = np.frombuffer(buf, dtype=np.uint8)
    return img


def golden_img(name: str) -> np.ndarray:
    with open(os.path.join(GOLDEN, name + ".bin"), "rb") as f:
        return np.frombuffer(f.read(), dtype=np.uint8).copy()


def case_ref_writelogentry():
    """db_test.go:182-229 TestLazyDB_WriteLogEntry: MaxLogFileSize 150, 32-B keys and values ->
    74-B entries at (1, 0), (1, 74), (2, 0). Here the three records are rewritten by a merge of
    archived file 0 into the empty active file 1."""
    val = bytes(range(65, 97))
    src = _log([dict(key=ref_key(i), value=val) for i in (1, 2, 3)])
    active = np.zeros(150, dtype=np.uint8)
    return [(src, 0, True), (active, 1, False)], dict(active_fid=1, active_off=0, max_file_size=150, now=NOW)


def case_ref_merge_shape():
    """db_test.go:64-109 TestLazyDB_Merge shape (strings only): MaxLogFileSize 500, Set(key1) x100
    then Set(key2) x100 with GetKey(32)-sized values; every archived file is merged."""
    recs = [dict(key=ref_key(1), value=ref_key(32))] * 100 + [dict(key=ref_key(2), value=ref_key(32))] * 100
    per = 500 // 74
    files = []
    for f in range(0, (len(recs) + per - 1) // per):
        files.append(_log(recs[f * per:(f + 1) * per], 500))
    last = len(files) - 1
    active_off = (len(recs) - last * per) * 74
    return ([(img, f, f != last) for f, img in enumerate(files)],
            dict(active_fid=last, active_off=active_off, max_file_size=500, now=NOW))


def case_generated(seed: int, n_files: int = 5, cap: int = 1 << 16, n_records: int = 900, max_file_size: int = 1 << 15,
                   p_delete: int = 50_000, p_expire: int = 50_000, ksize: int = 24, vsize: int = 40, targets=None):
    imgs, n, ends = coracle.gen_merge(n_files, cap, n_records, seed, ksize=ksize, vsize=vsize,
                                      p_delete_ppm=p_delete, p_expire_ppm=p_expire, now=NOW)
    if targets is None:
        targets = set(range(n_files - 1))
    last = n_files - 1
    files = [(imgs[i].copy(), 10 + i, i in targets) for i in range(n_files)]
    return files, dict(active_fid=10 + last, active_off=ends[last], max_file_size=max_file_size, now=NOW)


def case_golden_mix():
    """Golden fixtures as the files of one type: stat mix (SDelete / SListMeta), nil keys, empty
    values, non-canonical varints (re-encoded by EncodeEntry), big and binary values."""
    names = ["mixed_64k", "noncanonical", "noncanonical5", "zero_len_entries", "binary_values", "big_values",
             "ref_read_entries"]
    files = [(golden_img(nm), 3 + i, i != len(names) - 1) for i, nm in enumerate(names)]
    return files, dict(active_fid=3 + len(names) - 1, active_off=0, max_file_size=1 << 17, now=NOW)


def case_oversized():
    """Records larger than MaxLogFileSize: each roll-over check fires even at offset 0 (db.go:485)."""
    recs = [dict(key=b"k%d" % (i % 7), value=bytes([97 + i % 26]) * (30 + 17 * i)) for i in range(40)]
    return [(_log(recs[:20]), 1, True), (_log(recs[20:]), 2, True), (np.zeros(64, np.uint8), 3, False)], \
        dict(active_fid=3, active_off=10, max_file_size=200, now=NOW)


def case_hot_keys(seed: int):
    """Few distinct keys (incl. the nil key) rewritten many times across files, with SDeletes that are
    sometimes followed by a re-Put, expiring records, empty values and odd sizes."""
    import random
    rnd = random.Random(seed)
    keys = [b""] + [b"hot-%d" % i for i in range(9)] + [bytes([255 - i]) * (1 + i * 13) for i in range(6)]
    files = []
    for f in range(6):
        recs = []
        for _ in range(rnd.randint(20, 400)):
            k = rnd.choice(keys)
            if rnd.random() < 0.15:
                recs.append(dict(stat=1, key=k))
            else:
                exp = rnd.choice([0, 0, 0, NOW - 5, NOW + 5, NOW])
                recs.append(dict(stat=rnd.choice([0, 0, 0, 2]), expired_at=exp, tx_id=rnd.choice([0, 7, 1 << 40]),
                                 tx_stat=rnd.choice([0, 1, 2]), key=k,
                                 value=bytes(rnd.getrandbits(8) for _ in range(rnd.choice([0, 1, 15, 16, 17, 333])))))
        files.append(_log(recs, sum(len(coracle.encode_entry(**r)) for r in recs) + rnd.choice([0, 3, 40])))
    return [(img, 100 + f, f != 5) for f, img in enumerate(files)], \
        dict(active_fid=105, active_off=int(files[5].size), max_file_size=4096, now=NOW)


def case_tiny_entries():
    """15-B entries (5-B keys that repeat every 10 records, empty values): more records per file than
    the engine's first-pass slot of len/64 + 1024, so the scans are redone densely."""
    files = []
    for i in range(3):
        img, n, end = coracle.gen_log(200_000 + 999 * i, 20 + i, ksize=5, vsize=0)
        files.append((img, 1 + i, i < 2))
    return files, dict(active_fid=3, active_off=int(coracle.scan(files[2][0])[0].end_off), max_file_size=1 << 16,
                       now=NOW)


def case_prefix_keys():
    """Keys that are prefixes of one another, each followed by value bytes that continue the longer
    keys ("a" + value "aaa..." reads like the key "aaaa"), rewritten across files, with headers of
    every varint length (TTLs, tx ids): key identity must come from the key length, not the bytes."""
    keys = [b"a" * n for n in range(0, 40)] + [b"ab" * n for n in range(1, 9)]
    files = []
    for f in range(4):
        recs = []
        for i, k in enumerate(keys):
            if (i + f) % 3 == 0:
                continue
            recs.append(dict(key=k, value=b"a" * (5 + (i * 7 + f) % 50) + b"b" * f,
                             expired_at=[0, NOW + 100, NOW - 100, 1 << 40][(i + f) % 4],
                             tx_id=[0, 5, 1 << 30, (1 << 62) + 3][(i * 3 + f) % 4]))
        files.append(_log(recs))
    return [(img, 40 + f, f != 3) for f, img in enumerate(files)], \
        dict(active_fid=43, active_off=int(files[3].size), max_file_size=1 << 16, now=NOW)


def case_long_and_hot_keys():
    """Keys over 64 B that agree in their first 64 bytes (and more) and differ after them, keys of 63-65 B,
    and one key rewritten ~2,000 times across the files, among distinct keys (round 6)."""
    import random
    rnd = random.Random(77)
    longk = [b"L" * 64 + b"x" * j + b"%d" % i for i in range(6) for j in (0, 1, 40)]
    edge = [bytes([65 + i]) * n for i in range(3) for n in (63, 64, 65)]
    hot = b"hot-key"
    files = []
    for f in range(5):
        recs = []
        for r in range(900):
            u = rnd.random()
            if u < 0.45:
                k = hot
            elif u < 0.75:
                k = rnd.choice(longk + edge)
            else:
                k = b"k-%d-%d" % (f, r)
            if rnd.random() < 0.08:
                recs.append(dict(stat=1, key=k))
            else:
                recs.append(dict(key=k, value=bytes(rnd.getrandbits(8) for _ in range(rnd.choice([0, 9, 40]))),
                                 expired_at=rnd.choice([0, 0, 0, NOW - 1, NOW + 1])))
        files.append(_log(recs))
    return [(img, 10 + f, f != 4) for f, img in enumerate(files)], \
        dict(active_fid=14, active_off=int(files[4].size), max_file_size=1 << 16, now=NOW)


def case_crc_corrupt():
    return [(golden_img("mixed_64k"), 1, True), (golden_img("crc_corrupt"), 2, True),
            (np.zeros(64, np.uint8), 3, False)], dict(active_fid=3, active_off=0, max_file_size=1 << 20, now=NOW)


def small_cases():
    out = {"ref_writelogentry": case_ref_writelogentry(), "ref_merge_shape": case_ref_merge_shape(),
           "golden_mix": case_golden_mix(), "oversized": case_oversized(), "crc_corrupt": case_crc_corrupt()}
    for s in range(1, 5):
        out[f"gen{s}"] = case_generated(s)
    out["gen_no_targets"] = case_generated(7, targets=set())
    out["gen_all_but_one"] = case_generated(8, n_files=6, targets={0, 1, 3, 4}, max_file_size=5000)
    out["gen_mmap"] = (case_generated(9)[0], dict(case_generated(9)[1], io_type=1))
    for s in (1, 2, 3):
        out[f"hot_keys{s}"] = case_hot_keys(s)
    out["tiny_entries"] = case_tiny_entries()
    out["prefix_keys"] = case_prefix_keys()
    out["long_and_hot_keys"] = case_long_and_hot_keys()
    return out
