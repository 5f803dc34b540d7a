"""Host-side driver of the MI355X log-scan engine.

`Engine` owns one ldb_ctx (per device / per caller thread, like the reference's
one replay goroutine per value type, index.go:103-108) and scans log-file images
that live in HBM (torch uint8 tensors on a ROCm device) or in host memory.

PyTorch is only the device-memory / stream plumbing here: every byte of the scan
is done by the gfx950 kernels in liblazydb_gpu.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


class Engine:
    def __init__(self, device: int = 0):
        import torch
        if not torch.cuda.is_available():
            raise N.LdbError("no ROCm GPU visible: the log-scan engine has no CPU path")
        self.torch = torch
        self.device = device
        self.ctx = C.c_void_p()
        N.check(N.lib().ldb_ctx_create(device, C.byref(self.ctx)), "ldb_ctx_create")

    def close(self):
        if self.ctx:
            N.lib().ldb_ctx_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reserve(self, max_len: int):
        N.check(N.lib().ldb_ctx_reserve(self.ctx, max_len), "ldb_ctx_reserve")

    # ---------------------------------------------------------------- device-resident
    def alloc_out(self, cap: int, kind: int = N.TUPLE_INDEX):
        nbytes = cap * (16 if kind == N.TUPLE_INDEX else 48)
        return self.torch.empty(max(nbytes, 16), dtype=self.torch.uint8, device=f"cuda:{self.device}")

    def alloc_result(self):
        return self.torch.zeros(N.RESULT_BYTES, dtype=self.torch.uint8, device=f"cuda:{self.device}")

    def scan_dev_async(self, img, fid: int = 0, io_type: int = N.FILEIO, kind: int = N.TUPLE_INDEX, out=None,
                       cap: int = 0, result=None, serial: bool = False, stream=None):
        """Enqueue a scan of a device-resident uint8 tensor on `stream` (default: torch's current)."""
        t = self.torch
        assert img.dtype == t.uint8 and img.is_cuda and img.is_contiguous()
        if stream is None:
            stream = t.cuda.current_stream(img.device)
        fn = N.lib().ldb_scan_file_dev_serial if serial else N.lib().ldb_scan_file_dev
        rc = fn(self.ctx, C.c_void_p(img.data_ptr()), img.numel(), fid, io_type, kind,
                C.c_void_p(out.data_ptr()) if out is not None else None, cap,
                C.c_void_p(result.data_ptr()), C.c_void_p(stream.cuda_stream))
        N.check(rc, "ldb_scan_file_dev")

    def scan_dev(self, img, fid: int = 0, io_type: int = N.FILEIO, kind: int = N.TUPLE_INDEX, cap: int | None = None,
                 serial: bool = False):
        """Scan a device-resident image; returns (result dict, tuples as a numpy structured array)."""
        if cap is None:
            cap = img.numel() // 10 + 16
        out = self.alloc_out(cap, kind)
        res = self.alloc_result()
        self.scan_dev_async(img, fid, io_type, kind, out, cap, res, serial)
        r = N.ScanResult.from_buffer_copy(res.cpu().numpy().tobytes())
        n = min(r.n_entries, cap)
        dt = N.INDEX_TUPLE if kind == N.TUPLE_INDEX else N.ENTRY_TUPLE
        tuples = np.frombuffer(out[: n * dt.itemsize].cpu().numpy().tobytes(), dtype=dt) if n else np.zeros(0, dt)
        return r, tuples

    # ---------------------------------------------------------------- host memory
    def scan_host(self, img: np.ndarray, fid: int = 0, io_type: int = N.FILEIO, kind: int = N.TUPLE_INDEX,
                  cap: int | None = None):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        if cap is None:
            cap = img.size // 10 + 16
        dt = N.INDEX_TUPLE if kind == N.TUPLE_INDEX else N.ENTRY_TUPLE
        out = np.zeros(max(cap, 1), dtype=dt)
        res = N.ScanResult()
        N.check(N.lib().ldb_scan_file(self.ctx, img.ctypes.data if img.size else None, img.size, fid, io_type, kind,
                                      out.ctypes.data, cap, C.byref(res)), "ldb_scan_file")
        return res, out[: min(res.n_entries, cap)]

    def read_ceiling(self, d_img, iters: int = 20) -> float:
        """GB/s of a read-only reduction over the device image (the practical HBM-read ceiling)."""
        g = C.c_double()
        N.check(N.lib().ldb_read_ceiling(self.ctx, d_img.data_ptr(), d_img.numel(), iters, C.byref(g)), "read_ceiling")
        return g.value

    def timing(self, enable: int = -1):
        a, b, n = C.c_double(), C.c_double(), C.c_uint64()
        N.check(N.lib().ldb_kernel_timing(self.ctx, enable, C.byref(a), C.byref(b), C.byref(n)), "timing")
        return a.value, b.value, n.value
