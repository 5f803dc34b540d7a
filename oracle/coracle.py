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
                ("n_fast", C.c_uint32), ("reserved_", C.c_uint32)]


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
