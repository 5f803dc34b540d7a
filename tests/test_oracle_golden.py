"""The CPU oracles against the reference's own known-answer vectors and against each other.

Pins: logfile/log_entry_test.go:18-32 (EncodeEntry bytes), :57-69 (decodeHeader),
:93-104 (getEntryCrc), db_test.go:203-229 (entrySize 74, rollover at MaxLogFileSize=150),
logfile/log_file_test.go:38-116 (ReadLogEntry round trip + EOF one past the end).
"""
import random
import struct
import zlib

import numpy as np
import pytest

from oracle import coracle
from oracle import pyoracle as P

REF_ENCODE = [  # logfile/log_entry_test.go:18-32
    (dict(), [163, 161, 194, 177, 0, 0, 0, 0, 0, 0]),
    (dict(expired_at=1676969769, stat=2, tx_id=11111111, tx_stat=2, key=b"a", value=b"abc"),
     [17, 148, 49, 87, 2, 210, 156, 164, 191, 12, 142, 171, 204, 10, 4, 2, 6, 97, 97, 98, 99]),
    (dict(stat=1), [6, 114, 158, 122, 1, 0, 0, 0, 0, 0]),
]


@pytest.mark.parametrize("fields,want", REF_ENCODE)
def test_encode_entry_reference_vectors(fields, want):
    assert list(P.encode_entry(P.Entry(**fields))) == want
    assert list(coracle.encode_entry(**fields)) == want


def test_decode_header_reference_vectors():
    # logfile/log_entry_test.go:57-69
    e, n = P.decode_header(bytes([163, 161, 194, 177, 0, 0, 0, 0, 0, 0]))
    assert n == 10 and e.crc == 2982322595 and e.k_size == 0 and e.v_size == 0
    buf = bytes([43, 161, 225, 52, 2, 210, 156, 164, 191, 12, 142, 171, 204, 10, 2, 2, 6, 97, 97, 98, 99])
    e, n = P.decode_header(buf)
    assert n == 17
    assert (e.crc, e.expired_at, e.stat, e.tx_id, e.tx_stat, e.k_size, e.v_size) == \
        (887202091, 1676969769, 2, 11111111, 1, 1, 3)
    assert P.decode_header(bytes([105, 223, 34, 101])) == (None, 0)
    # C restatement on the same windows (padded to the 38-byte read window)
    h = coracle.Header()
    coracle.lib().ldbo_decode_header(np.frombuffer(buf + bytes(38 - len(buf)), np.uint8).ctypes.data, h)
    assert (h.crc, h.expired_at, h.stat, h.tx_id, h.tx_stat, h.k_size, h.v_size, h.size) == \
        (887202091, 1676969769, 2, 11111111, 1, 1, 3, 17)


def test_get_entry_crc_reference_vector():
    # logfile/log_entry_test.go:93-104: ChecksumIEEE(buf[4:]) then Update(Key) then Update(Value)
    buf = bytes([85, 205, 109, 118, 2, 210, 156, 164, 191, 12, 2, 6])
    c = zlib.crc32(buf[4:])
    c = zlib.crc32(b"a", c)
    c = zlib.crc32(b"abc", c)
    assert c == 3775086703
    assert coracle.crc32(b"abc", coracle.crc32(b"a", coracle.crc32(buf[4:]))) == 3775086703
    assert coracle.crc32(b"123456789") == 0xCBF43926


def test_entry_sizes_reference():
    # db_test.go:203-229: 32-B key + 32-B value -> 74; SURVEY: 64/256 -> 332
    assert len(P.encode_entry(P.Entry(key=b"k" * 32, value=b"v" * 32))) == 74
    assert len(P.encode_entry(P.Entry(key=b"k" * 64, value=b"v" * 256))) == 332


def test_varint_go_semantics():
    # Go 1.18 encoding/binary: short buffer -> (0,0); 11th byte -> (0,-11); 10th byte > 1 -> (0,-10)
    assert P.uvarint(b"\x80\x80") == (0, 0)
    assert P.uvarint(b"\xff" * 10 + b"\x01") == (0, -11)
    assert P.uvarint(b"\xff" * 9 + b"\x02") == (0, -10)
    assert P.uvarint(b"\xff" * 9 + b"\x01") == ((1 << 64) - 1, 10)
    for x in [0, 1, -1, 63, -64, 64, 1 << 40, -(1 << 63), (1 << 63) - 1]:
        enc = P.put_varint(x)
        assert P.varint(enc) == (x, len(enc))


def test_read_log_entry_roundtrip_reference():
    # logfile/log_file_test.go:38-116: 8 entries written back to back, read back, EOF one past the end
    meta_img = None
    from tests.golden.make_golden import ref_read_entries
    img = ref_read_entries()
    st, end, tup = P.scan(img)
    assert st == P.EOF_SENTINEL and len(tup) == 8
    assert [t[3] for t in tup] == [2, 1, 2, 0, 0, 0, 1, 1]
    assert [t[4] for t in tup] == [0, 0, 0, 2, 0, 2, 2, 2]
    assert [t[5] for t in tup] == [0, 0, 0, 0, 9, 4, 9, 9]
    del meta_img


def test_golden_fixtures_both_oracles(golden):
    meta, imgs = golden
    for m in meta:
        img = imgs[m["name"]]
        st, end, tup = P.scan(img, m["io_type"])
        assert (st, end) == (m["status"], m["end_off"]), m["name"]
        assert [list(t) for t in tup] == m["tuples"], m["name"]
        res, ct = coracle.scan(np.frombuffer(img, np.uint8), m["io_type"])
        assert (res.status, res.end_off, res.n_entries) == (m["status"], m["end_off"], len(m["tuples"])), m["name"]


@pytest.mark.parametrize("seed", range(6))
def test_c_and_python_oracles_agree_on_mutated_logs(seed):
    rng = random.Random(seed)
    img, n, end = coracle.gen_log(20000, seed, ksize=rng.choice([5, 16, 64]), vsize=rng.choice([0, 7, 100]))
    b = bytearray(img.tobytes())
    for _ in range(rng.randrange(0, 4)):
        b[rng.randrange(0, max(1, end))] = rng.randrange(256)
    for io in (0, 1):
        st, e, tup = P.scan(bytes(b), io)
        res, ct = coracle.scan(np.frombuffer(bytes(b), np.uint8), io, tuple_kind=0)
        assert (res.status, res.end_off, res.n_entries) == (st, e, len(tup))
        assert list(ct["pos"]) == [P.pack_pos(o, h, eh, s) for (o, h, eh, s, k, v) in tup]


def test_generator_config2_shape():
    # 64/256 entries -> 332 B each; 1 GiB -> 3 234 162 entries, 40 trailing zero bytes.
    img, n, end = coracle.gen_log(332 * 1000 + 40, 1)
    assert n == 1000 and end == 332000
    res, t = coracle.scan(img)
    assert res.status == P.EOF_SENTINEL and res.n_entries == 1000
    assert (1 << 30) // 332 == 3234162 and (1 << 30) - 3234162 * 332 == 40


def test_entry_tuple_kind_matches_index_kind():
    img, n, end = coracle.gen_log(50000, 3, ksize=10, vsize=50)
    r0, t0 = coracle.scan(img, tuple_kind=0)
    r1, t1 = coracle.scan(img, tuple_kind=1, fid=7)
    assert r0.n_entries == r1.n_entries == n
    assert np.array_equal(t0["pos"] & 0xFFFFFFFFFF, t1["offset"])
    assert np.all(t1["fid"] == 7) and np.array_equal(t0["k_size"], t1["k_size"])


def test_faithful_port_matches(tmp_path):
    img, n, end = coracle.gen_log(100000, 4, ksize=20, vsize=100)
    p = tmp_path / "log.strs.00000001"
    p.write_bytes(img.tobytes())
    import os
    fd = os.open(p, os.O_RDONLY)
    try:
        res, t = coracle.scan_faithful(fd, img.size, 0, 1, cap=n)
    finally:
        os.close(fd)
    r2, t2 = coracle.scan(img)
    assert (res.status, res.n_entries, res.end_off) == (r2.status, r2.n_entries, r2.end_off)
    assert np.array_equal(t["pos"], t2["pos"])


def test_crc_fold_and_table_formulations_equal_zlib():
    """The oracle's CRC-32 runs carry-less-multiply folding for spans of 64 B and more (the class of
    Go amd64 hash/crc32's IEEE path) and slicing-by-8 tables below that; both formulations must give
    zlib's CRC-32/IEEE on every length and alignment, including the check value of "123456789"."""
    import ctypes as C
    import zlib
    L = coracle.lib()
    L.ldbo_crc32_reg_tables.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
    L.ldbo_crc32_reg_tables.restype = C.c_uint32
    assert coracle.crc32(b"123456789") == 0xCBF43926
    rng = np.random.default_rng(7)
    buf = rng.integers(0, 256, 1 << 18, dtype=np.uint8)
    for t in range(1500):
        off = int(rng.integers(0, 64))
        n = int(rng.integers(0, 3000)) if t % 10 else int(rng.integers(0, 1 << 17))
        seg = buf[off:off + n]
        ptr = seg.ctypes.data if n else None
        want = zlib.crc32(seg.tobytes())
        assert L.ldbo_crc32_reg(0xFFFFFFFF, ptr, n) ^ 0xFFFFFFFF == want, (off, n)
        assert L.ldbo_crc32_reg_tables(0xFFFFFFFF, ptr, n) ^ 0xFFFFFFFF == want, (off, n)
