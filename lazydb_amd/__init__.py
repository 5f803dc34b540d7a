"""lazydb_amd — MI355X-native decode/verify engine for LazyDB bitcask log files.

Replaces the per-entry body of LazyDB's replay (logfile/log_file.go:116-145
ReadLogEntry + logfile/log_entry.go codec, driven by index.go:84-95) with a
parallel gfx950 scan behind the C ABI in include/lazydb_gpu.h.
"""
from ._native import (EOF_KV, EOF_SENTINEL, EOF_WINDOW, ERR_CAPACITY, ERR_CRC, ERR_MALFORMED, FILEIO, MMAP,  # noqa
                      TUPLE_ENTRY, TUPLE_INDEX, INDEX_TUPLE, ENTRY_TUPLE, LdbError, ScanResult, status_str)
from .build import build_all  # noqa: F401

__all__ = ["Engine", "build_all", "status_str"]


def __getattr__(name):
    if name == "Engine":
        from .engine import Engine
        return Engine
    raise AttributeError(name)
