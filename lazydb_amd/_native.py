"""ctypes binding of liblazydb_gpu.so (the C ABI in include/lazydb_gpu.h).

The library is the product: hand-written gfx950 kernels behind a C ABI. There is
no CPU fallback — if the library is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LAZYDB_GPU_LIB") or os.path.join(HERE, "_lib", "liblazydb_gpu.so")

LDB_OK = 0
EOF_WINDOW, EOF_SENTINEL, EOF_KV = 1, 2, 3
ERR_CRC, ERR_MALFORMED, ERR_CAPACITY, ERR_ARG, ERR_HIP, ERR_NOMEM, ERR_INTERNAL = -1, -2, -3, -4, -5, -6, -7
FILEIO, MMAP = 0, 1
TUPLE_INDEX, TUPLE_ENTRY = 0, 1

INDEX_TUPLE = np.dtype([("pos", "<u8"), ("k_size", "<u4"), ("v_size", "<u4")])
ENTRY_TUPLE = np.dtype([("offset", "<u8"), ("expired_at", "<i8"), ("tx_id", "<u8"), ("crc", "<u4"),
                        ("k_size", "<u4"), ("v_size", "<u4"), ("tx_stat", "<u2"), ("stat", "u1"),
                        ("hdr_size", "u1"), ("enc_hdr_size", "u1"), ("pad_", "u1", (3,)), ("fid", "<u4")])


class ScanResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("fid", C.c_uint32), ("n_entries", C.c_uint64), ("end_off", C.c_uint64),
                ("n_repairs", C.c_uint32), ("n_regions", C.c_uint32),
                ("n_fast", C.c_uint32), ("n_broken", C.c_uint32), ("n_run", C.c_uint64),
                ("n_sweep", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class MergeFile(C.Structure):
    _fields_ = [("d_image", C.c_void_p), ("len", C.c_uint64), ("fid", C.c_uint32), ("is_target", C.c_uint32)]


class MergeResult(C.Structure):
    _fields_ = [("status", C.c_int32), ("bad_file", C.c_int32), ("n_records", C.c_uint64), ("n_live", C.c_uint64),
                ("n_emit", C.c_uint64), ("emit_bytes", C.c_uint64), ("end_fid", C.c_uint32),
                ("n_segments", C.c_uint32), ("end_off", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


MERGE_POS = np.dtype([("offset", "<u8"), ("fid", "<u4"), ("entry_size", "<u4"), ("src_offset", "<u8"),
                      ("src_file", "<u4"), ("reserved_", "<u4")])
MERGE_SEGMENT = np.dtype([("fid", "<u4"), ("reserved_", "<u4"), ("file_off", "<u8"), ("stream_off", "<u8"),
                          ("n_bytes", "<u8")])
MERGE_FILE_STAT = np.dtype([("status", "<i4"), ("fid", "<u4"), ("n_entries", "<u8"), ("end_off", "<u8"),
                            ("live_count", "<u8"), ("live_bytes", "<u8")])
ENCODE_ITEM = np.dtype([("key_off", "<u8"), ("value_off", "<u8"), ("k_size", "<u4"), ("v_size", "<u4"),
                        ("expired_at", "<i8"), ("tx_id", "<u8"), ("tx_stat", "<u2"), ("stat", "u1"),
                        ("pad_", "u1", (5,))])
assert C.sizeof(MergeFile) == 24 and C.sizeof(MergeResult) == 56 and ENCODE_ITEM.itemsize == 48
assert MERGE_POS.itemsize == 32 and MERGE_SEGMENT.itemsize == 32 and MERGE_FILE_STAT.itemsize == 40
ROUTE_REC = np.dtype([("hash", "<u8"), ("seq", "<u4"), ("k_size", "<u4"), ("key_off", "<u8")])   # ldb_route_rec
assert ROUTE_REC.itemsize == 24

RESULT_BYTES = C.sizeof(ScanResult)
assert RESULT_BYTES == 56

_lib = None


class LdbError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise LdbError(f"{LIB_PATH} is missing: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
        L = C.CDLL(LIB_PATH)
        vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int
        L.ldb_abi_version.restype = i32
        L.ldb_status_str.argtypes = [i32]
        L.ldb_status_str.restype = C.c_char_p
        L.ldb_ctx_create.argtypes = [i32, C.POINTER(vp)]
        L.ldb_ctx_destroy.argtypes = [vp]
        L.ldb_ctx_reserve.argtypes = [vp, u64]
        L.ldb_workspace_bytes.argtypes = [u64]
        L.ldb_workspace_bytes.restype = u64
        L.ldb_scan_file_dev.argtypes = [vp, vp, u64, u32, i32, i32, vp, u64, vp, vp]
        L.ldb_scan_file_dev_serial.argtypes = [vp, vp, u64, u32, i32, i32, vp, u64, vp, vp]
        L.ldb_scan_file.argtypes = [vp, vp, u64, u32, i32, i32, vp, u64, C.POINTER(ScanResult)]
        L.ldb_scan_file_count.argtypes = [vp, vp, u64, u32, i32, i32, C.POINTER(ScanResult)]
        L.ldb_scan_copy_out.argtypes = [vp, vp, u64, C.POINTER(u64)]
        L.ldb_scan_files_dev.argtypes = [vp, i32, vp, vp, vp, i32, i32, vp, vp, vp, vp]
        L.ldb_kernel_timing.argtypes = [vp, i32, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(u64)]
        L.ldb_kernel_timing_split.argtypes = [vp, i32, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                              C.POINTER(C.c_double), C.POINTER(u64)]
        L.ldb_kernel_timing_split.restype = i32
        if hasattr(L, "ldb_kernel_timing_tail"):   # absent from A/B builds of older revisions
            L.ldb_kernel_timing_tail.argtypes = [vp, C.POINTER(C.c_double), i32]
            L.ldb_kernel_timing_tail.restype = i32
        if hasattr(L, "ldb_kernel_timing_sweep"):
            L.ldb_kernel_timing_sweep.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double)]
            L.ldb_kernel_timing_sweep.restype = i32
        for fn in ("ldb_ctx_create", "ldb_ctx_destroy", "ldb_ctx_reserve", "ldb_scan_file_dev",
                   "ldb_scan_file_dev_serial", "ldb_scan_file", "ldb_scan_files_dev", "ldb_kernel_timing"):
            getattr(L, fn).restype = i32
        if hasattr(L, "ldb_read_ceiling"):   # absent from A/B builds of older revisions (tools/build_variants.py)
            L.ldb_read_ceiling.argtypes = [vp, vp, u64, i32, C.POINTER(C.c_double)]
            L.ldb_read_ceiling.restype = i32
        if hasattr(L, "ldb_merge_files_dev"):   # absent from A/B builds of older revisions
            L.ldb_merge_files_dev.argtypes = [vp, i32, vp, i32, u32, u64, u64, C.c_int64, vp, u64, vp, u64, vp, u32,
                                              vp, u64, vp, C.POINTER(MergeResult), vp]
            L.ldb_merge_files_dev.restype = i32
            L.ldb_merge_timing.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]
            L.ldb_merge_timing.restype = i32
        if hasattr(L, "ldb_host_register"):
            L.ldb_host_register.argtypes = [vp, vp, u64]
            L.ldb_host_register.restype = i32
            L.ldb_host_unregister.argtypes = [vp, vp]
            L.ldb_host_unregister.restype = i32
        if hasattr(L, "ldb_merge_repack_dev"):
            L.ldb_merge_repack_dev.argtypes = [vp, u64, vp, vp, u32, u64, u64, vp, u32, vp, vp]
            L.ldb_merge_repack_dev.restype = i32
        if hasattr(L, "ldb_merge_route_dev"):
            L.ldb_merge_route_dev.argtypes = [vp, i32, vp, i32, u32, vp, u64, vp, u64, vp, C.POINTER(MergeResult), vp]
            L.ldb_merge_route_dev.restype = i32
            L.ldb_merge_resolve_dev.argtypes = [vp, u64, vp, vp, vp, vp, vp]
            L.ldb_merge_resolve_dev.restype = i32
            L.ldb_merge_apply_dev.argtypes = [vp, i32, vp, i32, vp, u32, u64, u64, C.c_int64, vp, u64, vp, u64, vp,
                                              u32, vp, u64, vp, C.POINTER(MergeResult), vp]
            L.ldb_merge_apply_dev.restype = i32
        if hasattr(L, "ldb_encode_entries_dev"):
            L.ldb_encode_entries_dev.argtypes = [vp, u64, vp, vp, u32, u64, u64, vp, u64, vp, u64, vp, u32,
                                                 C.POINTER(MergeResult), vp]
            L.ldb_encode_entries_dev.restype = i32
        # (an A/B build of an older revision, LAZYDB_GPU_LIB, may be one ABI behind)
        if L.ldb_abi_version() != 4 and not (os.environ.get("LAZYDB_GPU_LIB") and L.ldb_abi_version() == 3):
            raise LdbError("liblazydb_gpu ABI version mismatch")
        _lib = L
    return _lib


EXPORTS = ("ldb_abi_version", "ldb_status_str", "ldb_ctx_create", "ldb_ctx_destroy", "ldb_ctx_reserve",
           "ldb_workspace_bytes", "ldb_scan_file_dev", "ldb_scan_file", "ldb_scan_file_count", "ldb_scan_copy_out",
           "ldb_scan_files_dev",
           "ldb_scan_file_dev_serial", "ldb_kernel_timing", "ldb_kernel_timing_split", "ldb_kernel_timing_tail",
           "ldb_kernel_timing_sweep",
           "ldb_read_ceiling", "ldb_merge_files_dev",
           "ldb_merge_timing", "ldb_encode_entries_dev", "ldb_merge_repack_dev", "ldb_host_register", "ldb_host_unregister",
           "ldb_merge_route_dev", "ldb_merge_resolve_dev", "ldb_merge_apply_dev")


def status_str(s: int) -> str:
    return lib().ldb_status_str(s).decode()


def check(rc: int, what: str):
    if rc != LDB_OK:
        raise LdbError(f"{what}: {status_str(rc)} ({rc})")
