"""ctypes binding of oracle/_build/libldb_oracle.so (the C restatement).

TEST INFRASTRUCTURE ONLY — loaded by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py; never by the lazydb_amd product path.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libldb_oracle.so")


class ScanResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("fid", C.c_uint32), ("n_entries", C.c_uint64), ("end_off", C.c_uint64),
                ("n_repairs", C.c_uint32), ("n_regions", C.c_uint32),
                ("n_fast", C.c_uint32), ("reserved_", C.c_uint32), ("n_run", C.c_uint64),
                ("n_sweep", C.c_uint64)]


class Header(C.Structure):
    _fields_ = [("crc", C.c_uint32), ("stat", C.c_uint8), ("expired_at", C.c_int64), ("tx_id", C.c_uint64),
                ("tx_stat", C.c_uint16), ("k_size", C.c_uint32), ("v_size", C.c_uint32), ("size", C.c_int32),
                ("enc_size", C.c_int32)]


INDEX_TUPLE = np.dtype([("pos", "<u8"), ("k_size", "<u4"), ("v_size", "<u4")])
ENTRY_TUPLE = np.dtype([("offset", "<u8"), ("expired_at", "<i8"), ("tx_id", "<u8"), ("crc", "<u4"),
                        ("k_size", "<u4"), ("v_size", "<u4"), ("tx_stat", "<u2"), ("stat", "u1"),
                        ("hdr_size", "u1"), ("enc_hdr_size", "u1"), ("pad_", "u1", (3,)), ("fid", "<u4")])
assert INDEX_TUPLE.itemsize == 16 and ENTRY_TUPLE.itemsize == 48

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = C.CDLL(_SO)
        u8p = C.POINTER(C.c_uint8)
        L.ldbo_crc32_update.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.ldbo_crc32_update.restype = C.c_uint32
        L.ldbo_crc32_reg.argtypes = [C.c_uint32, C.c_void_p, C.c_size_t]
        L.ldbo_crc32_reg.restype = C.c_uint32
        L.ldbo_decode_header.argtypes = [C.c_void_p, C.POINTER(Header)]
        L.ldbo_read_log_entry.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint64, C.POINTER(Header),
                                          C.POINTER(C.c_uint64)]
        L.ldbo_scan.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_int, C.c_void_p, C.c_uint64,
                                C.POINTER(ScanResult)]
        L.ldbo_scan_faithful.argtypes = [C.c_int, C.c_uint64, C.c_int, C.c_uint32, C.c_void_p, C.c_uint64,
                                         C.POINTER(ScanResult)]
        L.ldbo_encode_entry.argtypes = [C.c_uint8, C.c_int64, C.c_uint64, C.c_uint16, C.c_void_p, C.c_uint32,
                                        C.c_void_p, C.c_uint32, C.c_void_p]
        L.ldbo_encode_entry.restype = C.c_size_t
        L.ldbo_gen_log.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint32, C.c_int, C.c_double,
                                   C.c_uint32, C.c_uint64, C.POINTER(C.c_uint64)]
        L.ldbo_gen_log.restype = C.c_uint64
        del u8p
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def crc32(data: bytes, crc: int = 0) -> int:
    b = np.frombuffer(data, dtype=np.uint8)
    return lib().ldbo_crc32_update(crc, _ptr(b) if len(b) else None, len(b))


def encode_entry(stat=0, expired_at=0, tx_id=0, tx_stat=0, key=b"", value=b"") -> bytes:
    out = np.zeros(38 + len(key) + len(value), dtype=np.uint8)
    k = np.frombuffer(key, dtype=np.uint8) if key else None
    v = np.frombuffer(value, dtype=np.uint8) if value else None
    n = lib().ldbo_encode_entry(stat, expired_at, tx_id, tx_stat, _ptr(k) if k is not None else None, len(key),
                                _ptr(v) if v is not None else None, len(value), _ptr(out))
    return out[:n].tobytes()


def scan(img: np.ndarray, io_type: int = 0, fid: int = 0, tuple_kind: int = 0, cap: int | None = None):
    """index.go replay over a uint8 image. Returns (ScanResult, tuples ndarray)."""
    img = np.ascontiguousarray(img, dtype=np.uint8)
    res = ScanResult()
    if cap is None:
        lib().ldbo_scan(_ptr(img), img.size, io_type, fid, tuple_kind, None, 0, C.byref(res))
        cap = res.n_entries
    dt = INDEX_TUPLE if tuple_kind == 0 else ENTRY_TUPLE
    out = np.zeros(max(int(cap), 1), dtype=dt)
    lib().ldbo_scan(_ptr(img), img.size, io_type, fid, tuple_kind, _ptr(out), int(cap), C.byref(res))
    return res, out[:min(int(cap), res.n_entries)]


def scan_faithful(fd: int, length: int, io_type: int = 0, fid: int = 0, cap: int = 0):
    res = ScanResult()
    out = np.zeros(max(cap, 1), dtype=INDEX_TUPLE)
    lib().ldbo_scan_faithful(fd, length, io_type, fid, _ptr(out) if cap else None, cap, C.byref(res))
    return res, out[:min(cap, res.n_entries)]


def gen_log(cap_bytes: int, seed: int, ksize: int = 64, vsize: int = 256, value_mode: int = 0,
            zipf_s: float = 1.1, zipf_max: int = 4096, max_entries: int = (1 << 63), img: np.ndarray | None = None):
    """Synthetic LazyDB log (writeLogEntry format, zero-preallocated). Returns (img, n, end_off)."""
    if img is None:
        img = np.zeros(cap_bytes, dtype=np.uint8)
    end = C.c_uint64(0)
    n = lib().ldbo_gen_log(_ptr(img), cap_bytes, seed, ksize, vsize, value_mode, zipf_s, zipf_max, max_entries,
                           C.byref(end))
    return img, int(n), int(end.value)


def gen_bench_log(cap_bytes: int = 512 << 20, seed: int = 1, n_entries: int = 500_000, vsize: int = 512,
                  img: np.ndarray | None = None):
    """The reference benchmark's log (bench/db_bench_test.go:17-36): n Sets of "bench_test_key_<i>" with
    512-B alphabet values in one zero-preallocated file of cap_bytes (Mmap: MaxLogFileSize).
    Returns (img, n, end_off)."""
    L = lib()
    if not hasattr(L.ldbo_gen_bench_log, "_typed"):
        L.ldbo_gen_bench_log.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                         C.POINTER(C.c_uint64)]
        L.ldbo_gen_bench_log.restype = C.c_uint64
        L.ldbo_gen_bench_log._typed = True
    if img is None:
        img = np.zeros(cap_bytes, dtype=np.uint8)
    end = C.c_uint64(0)
    n = L.ldbo_gen_bench_log(_ptr(img), cap_bytes, seed, n_entries, vsize, C.byref(end))
    return img, int(n), int(end.value)


def gen_writer_log(cap_bytes: int, seed: int, max_entries: int = (1 << 63), now: int = 1_760_000_000,
                   key_space: int = 1_000_000, vmax: int = 4096, p_setex: int = 100, p_del: int = 100,
                   p_tx: int = 100, img: np.ndarray | None = None):
    """Writer-realistic string log (Set / SetEX / Delete / Tx.Commit interleaved, str.go, tx.go).
    p_* in parts per 1000. Returns (img, n, end_off)."""
    L = lib()
    if not hasattr(L.ldbo_gen_writer_log, "_typed"):
        L.ldbo_gen_writer_log.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int64, C.c_uint32,
                                          C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint64)]
        L.ldbo_gen_writer_log.restype = C.c_uint64
        L.ldbo_gen_writer_log._typed = True
    if img is None:
        img = np.zeros(cap_bytes, dtype=np.uint8)
    end = C.c_uint64(0)
    n = L.ldbo_gen_writer_log(_ptr(img), cap_bytes, seed, max_entries, now, key_space, vmax, p_setex, p_del, p_tx,
                              C.byref(end))
    return img, int(n), int(end.value)


# ---------------------------------------------------------------- merge / GC (db.go:243-265, 383-427, 473-523)
class MergeFile(C.Structure):
    _fields_ = [("d_image", C.c_void_p), ("len", C.c_uint64), ("fid", C.c_uint32), ("is_target", C.c_uint32)]


class MergeResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("bad_file", C.c_int32), ("n_records", C.c_uint64), ("n_live", C.c_uint64),
                ("n_emit", C.c_uint64), ("emit_bytes", C.c_uint64), ("end_fid", C.c_uint32),
                ("n_segments", C.c_uint32), ("end_off", C.c_uint64)]


MERGE_POS = np.dtype([("offset", "<u8"), ("fid", "<u4"), ("entry_size", "<u4"), ("src_offset", "<u8"),
                      ("src_file", "<u4"), ("reserved_", "<u4")])
MERGE_SEGMENT = np.dtype([("fid", "<u4"), ("reserved_", "<u4"), ("file_off", "<u8"), ("stream_off", "<u8"),
                          ("n_bytes", "<u8")])
MERGE_FILE_STAT = np.dtype([("status", "<i4"), ("fid", "<u4"), ("n_entries", "<u8"), ("end_off", "<u8"),
                            ("live_count", "<u8"), ("live_bytes", "<u8")])


def merge(files, active_fid: int, active_off: int, max_file_size: int, now: int, io_type: int = 0):
    """C restatement of Merge over host images. files: list of (uint8 ndarray, fid, is_target).
    Returns (MergeResult, stream bytes ndarray, pos, segments, live flags, per-file stats)."""
    L = lib()
    if not hasattr(L.ldbo_merge, "_typed"):
        L.ldbo_merge.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_uint32, C.c_uint64, C.c_uint64, C.c_int64,
                                 C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint32, C.c_void_p,
                                 C.c_uint64, C.c_void_p, C.POINTER(MergeResult)]
        L.ldbo_merge._typed = True
    imgs = [np.ascontiguousarray(f[0], dtype=np.uint8) for f in files]
    arr = (MergeFile * max(len(files), 1))()
    tgt = 0
    tot = 0
    for i, (img, (_, fid, tg)) in enumerate(zip(imgs, files)):
        arr[i].d_image = _ptr(img) if img.size else None
        arr[i].len = img.size
        arr[i].fid = fid
        arr[i].is_target = 1 if tg else 0
        tot += img.size
        tgt += img.size if tg else 0
    stream = np.zeros(max(tgt, 1), dtype=np.uint8)
    pos_cap = tgt // 10 + 2
    pos = np.zeros(pos_cap, dtype=MERGE_POS)
    seg_cap = 1 << 16
    segs = np.zeros(seg_cap, dtype=MERGE_SEGMENT)
    live_cap = tot // 10 + 2
    live = np.zeros(live_cap, dtype=np.uint8)
    stats = np.zeros(max(len(files), 1), dtype=MERGE_FILE_STAT)
    res = MergeResult()
    L.ldbo_merge(len(files), C.addressof(arr), io_type, active_fid, active_off, max_file_size, now, _ptr(stream),
                 stream.size, _ptr(pos), pos_cap, _ptr(segs), seg_cap, _ptr(live), live_cap, _ptr(stats), C.byref(res))
    return (res, stream[: res.emit_bytes], pos[: res.n_emit], segs[: res.n_segments], live[: res.n_records],
            stats[: len(files)])


def gen_merge(n_files: int, cap_bytes: int, n_records: int, seed: int, ksize: int = 64, vsize: int = 256,
              p_delete_ppm: int = 0, p_expire_ppm: int = 0, now: int = 1_700_000_000):
    """Config-5-shaped merge set: consecutive files of cap_bytes, every key written twice.
    Returns (list of per-file uint8 arrays (views of one buffer), records written, end offsets)."""
    L = lib()
    if not hasattr(L.ldbo_gen_merge, "_typed"):
        L.ldbo_gen_merge.argtypes = [C.c_void_p, C.c_uint32, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32,
                                     C.c_uint32, C.c_uint32, C.c_uint32, C.c_int64, C.c_void_p]
        L.ldbo_gen_merge.restype = C.c_uint64
        L.ldbo_gen_merge._typed = True
    buf = np.zeros(n_files * cap_bytes, dtype=np.uint8)
    ends = np.zeros(n_files, dtype=np.uint64)
    n = L.ldbo_gen_merge(_ptr(buf), n_files, cap_bytes, n_records, seed, ksize, vsize, p_delete_ppm, p_expire_ppm,
                         now, _ptr(ends))
    return [buf[i * cap_bytes:(i + 1) * cap_bytes] for i in range(n_files)], int(n), [int(e) for e in ends]
