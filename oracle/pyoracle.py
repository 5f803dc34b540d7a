"""Pure-Python restatement of LazyDB's log codec and replay scan.

TEST INFRASTRUCTURE ONLY: an independent second oracle (CRC from zlib, varints
written from the Go spec) used to cross-check oracle/ldb_oracle.c and to write
the small golden fixtures under tests/golden/.  Only tests/, smoke() and
bench.py's cpu_baseline may use anything under oracle/.

Parity pinning: the Go reference cannot be built or run here (no Go
toolchain; mmap/mmap.go:24 `msync` vs mmap/mmap_linux.go:75 `mSync`).  This
module reproduces the reference's literal vectors in
logfile/log_entry_test.go:18-32, 57-69, 93-104 (see tests/test_oracle_golden.py).
"""
from __future__ import annotations

import struct
import zlib
from dataclasses import dataclass

MAX_HEADER = 38  # logfile/log_entry.go:32

FILEIO, MMAP = 0, 1  # logfile/log_file.go:35-41

OK, EOF_WINDOW, EOF_SENTINEL, EOF_KV = 0, 1, 2, 3
ERR_CRC, ERR_MALFORMED = -1, -2


def uvarint(buf: bytes) -> tuple[int, int]:
    """encoding/binary.Uvarint (Go 1.18)."""
    x = 0
    s = 0
    for i, b in enumerate(buf):
        if i == 10:
            return 0, -(i + 1)
        if b < 0x80:
            if i == 9 and b > 1:
                return 0, -(i + 1)
            return x | (b << s), i + 1
        x |= (b & 0x7F) << s
        s += 7
    return 0, 0


def varint(buf: bytes) -> tuple[int, int]:
    """encoding/binary.Varint: zigzag over Uvarint."""
    ux, n = uvarint(buf)
    x = ux >> 1
    if ux & 1:
        x = ~x
    # int64(ux >> 1) is always non-negative before the complement
    return x, n


def put_varint(x: int) -> bytes:
    """encoding/binary.PutVarint for an int64 x."""
    x &= (1 << 64) - 1
    sx = x - (1 << 64) if x >> 63 else x
    ux = (x << 1) & ((1 << 64) - 1)
    if sx < 0:
        ux = (~ux) & ((1 << 64) - 1)
    out = bytearray()
    while ux >= 0x80:
        out.append((ux & 0x7F) | 0x80)
        ux >>= 7
    out.append(ux)
    return bytes(out)


def _i64(x: int) -> int:
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


@dataclass
class Entry:
    """logfile.LogEntry (log_entry.go:35-45)."""

    crc: int = 0
    expired_at: int = 0
    stat: int = 0
    tx_id: int = 0
    tx_stat: int = 0
    k_size: int = 0
    v_size: int = 0
    key: bytes = b""
    value: bytes = b""


def encode_entry(e: Entry) -> bytes:
    """logfile.EncodeEntry (log_entry.go:48-78)."""
    hdr = bytearray(5)
    hdr[4] = e.stat & 0xFF
    hdr += put_varint(e.expired_at)
    hdr += put_varint(_i64(e.tx_id))
    hdr += put_varint(e.tx_stat & 0xFFFF)
    hdr += put_varint(len(e.key))
    hdr += put_varint(len(e.value))
    buf = bytes(hdr) + e.key + e.value
    crc = zlib.crc32(buf[4:]) & 0xFFFFFFFF
    return struct.pack("<I", crc) + buf[4:]


def decode_header(win: bytes):
    """logfile.decodeHeader (log_entry.go:81-107). Returns (Entry, size) or None if Go panics."""
    if len(win) <= 4:
        return None, 0
    e = Entry()
    e.crc = struct.unpack_from("<I", win, 0)[0]
    e.stat = win[4]
    off = 5
    vals = []
    for _ in range(5):
        if off < 0:
            return "panic", 0
        v, n = varint(win[off:])
        vals.append(v)
        off += n
    e.expired_at = _i64(vals[0])
    e.tx_id = vals[1] & ((1 << 64) - 1)
    e.tx_stat = vals[2] & 0xFFFF
    e.k_size = vals[3] & 0xFFFFFFFF
    e.v_size = vals[4] & 0xFFFFFFFF
    return e, off


def enc_header_size(e: Entry) -> int:
    return 5 + len(put_varint(e.expired_at)) + len(put_varint(_i64(e.tx_id))) + len(put_varint(e.tx_stat)) + \
        len(put_varint(e.k_size)) + len(put_varint(e.v_size))


def _read_eof(length: int, io_type: int, off: int, n: int) -> bool:
    if io_type == MMAP:  # iocontroller/mmap.go:48
        return off < 0 or off >= length or off + n >= length
    return off + n > length  # os.File.ReadAt short read -> io.EOF


def read_log_entry(img: bytes, io_type: int, off: int):
    """(*LogFile).ReadLogEntry (log_file.go:116-145): (status, Entry|None, size, hdr_size)."""
    length = len(img)
    if _read_eof(length, io_type, off, MAX_HEADER):
        return EOF_WINDOW, None, 0, 0
    e, size = decode_header(img[off:off + MAX_HEADER])
    if e == "panic":
        return ERR_MALFORMED, None, 0, 0
    if e.crc == 0 and e.k_size == 0 and e.v_size == 0:
        return EOF_SENTINEL, None, 0, 0
    kv = e.k_size + e.v_size
    if e.k_size > 0 or e.v_size > 0:
        at = off + size
        if io_type == FILEIO and at < 0:
            return ERR_MALFORMED, None, 0, 0
        if _read_eof(length, io_type, at, kv):
            return EOF_KV, None, 0, 0
        e.key = bytes(img[at:at + e.k_size])
        e.value = bytes(img[at + e.k_size:at + kv])
    if size < 0:
        return ERR_MALFORMED, None, 0, 0
    crc = 0
    if size > 4:
        crc = zlib.crc32(bytes(img[off + 4:off + size]))
        crc = zlib.crc32(e.key, crc)
        crc = zlib.crc32(e.value, crc)
    if crc != e.crc:
        return ERR_CRC, None, 0, 0
    return OK, e, size + kv, size


def scan(img: bytes, io_type: int = FILEIO, fid: int = 0):
    """The replay loop of index.go:84-95. Returns (status, end_off, tuples) with
    tuples = [(offset, hdr_size, enc_hdr_size, stat, k_size, v_size)]."""
    off = 0
    out = []
    while True:
        st, e, es, h = read_log_entry(img, io_type, off)
        if st != OK:
            return st, off, out
        out.append((off, h, enc_header_size(e), e.stat, e.k_size, e.v_size))
        off += es


def pack_pos(off: int, h: int, eh: int, stat: int) -> int:
    return (off & 0xFFFFFFFFFF) | ((h & 0x3F) << 40) | ((eh & 0x3F) << 46) | ((stat & 0xFF) << 52)


def merge(files, active_fid: int, active_off: int, max_file_size: int, now: int, io_type: int = FILEIO):
    """Merge of the string type, written as the reference runs it (pure Python; small inputs only).

    files: [(image bytes, fid, is_target)] ascending fid. Replays every file into a dict index
    (index.go:68-95, buildStrIndex :15-26: SDelete -> Delete, else Put), then for each target file
    in ascending fid runs db.go:383-427 (skip SDelete :403, skip expired :406-409, mergeStr :255 ->
    writeLogEntry db.go:473-523 with EncodeEntry and the rollover rule, then updateIndexTree).
    Returns dict(status, bad_file, stream, pos [(fid, off, size, src_off, src_file)],
    segments [(fid, file_off, stream_off, n_bytes)], live [0/1 per record], end_fid, end_off)."""
    recs = []   # (file index, offset, Entry)
    for fi, (img, fid, _) in enumerate(files):
        off = 0
        while True:
            st, e, es, _h = read_log_entry(img, io_type, off)
            if st != OK:
                break
            recs.append((fi, off, e))
            off += es
        if st < 0:
            return {"status": st, "bad_file": fi}
    index = {}
    for i, (fi, off, e) in enumerate(recs):
        if e.stat == 1:
            index.pop(e.key, None)   # idxTree.Delete
        else:
            index[e.key] = (fi, off)   # idxTree.Put
    live = [1 if index.get(e.key) == (fi, off) else 0 for (fi, off, e) in recs]
    fid, foff = active_fid, active_off
    stream = bytearray()
    pos, segs = [], []
    for (fi, off, e) in recs:
        if not files[fi][2]:
            continue
        if e.stat == 1:
            continue
        if e.expired_at != 0 and e.expired_at <= now:
            continue
        if index.get(e.key) != (fi, off):
            continue
        buf = encode_entry(e)
        if foff + len(buf) > max_file_size:
            fid, foff = fid + 1, 0
        if not segs or segs[-1][0] != fid or segs[-1][1] + segs[-1][3] != foff:
            segs.append([fid, foff, len(stream), 0])
        segs[-1][3] += len(buf)
        pos.append((fid, foff, len(buf), off, fi))
        index[e.key] = ("new", fid, foff)   # updateIndexTree with the new ValuePos
        stream += buf
        foff += len(buf)
    return {"status": 0, "bad_file": -1, "stream": bytes(stream), "pos": pos, "segments": [tuple(s) for s in segs],
            "live": live, "end_fid": fid, "end_off": foff}


def write_entries(entries, active_fid: int, active_off: int, max_file_size: int):
    """A transaction commit's writeLogEntry loop (tx.go:156-206 -> db.go:473-523) over Entry objects:
    EncodeEntry, rollover to fid+1 when Offset + size > MaxLogFileSize, append. Returns
    (stream bytes, [(fid, offset, size)], segments [(fid, file_off, stream_off, n_bytes)], end_fid, end_off)."""
    fid, off = active_fid, active_off
    stream = bytearray()
    pos, segs = [], []
    for e in entries:
        buf = encode_entry(e)
        if off + len(buf) > max_file_size:
            fid, off = fid + 1, 0
        if not segs or segs[-1][0] != fid or segs[-1][1] + segs[-1][3] != off:
            segs.append([fid, off, len(stream), 0])
        segs[-1][3] += len(buf)
        pos.append((fid, off, len(buf)))
        stream += buf
        off += len(buf)
    return bytes(stream), pos, [tuple(x) for x in segs], fid, off
