"""CPU-only checks of the product library and of the engine algorithm (no GPU needed).

* liblazydb_gpu.so loads and exports every symbol include/lazydb_gpu.h declares;
* the engine's own phase functions, run by the CPU wave emulator (tests/emu), equal
  the oracle on the golden fixtures and on randomized / mutated logs.
"""
import ctypes as C
import os
import random
import re

import numpy as np
import pytest

from oracle import coracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_header_symbols():
    from lazydb_amd import _native as N
    L = N.lib()
    with open(os.path.join(ROOT, "include", "lazydb_gpu.h")) as f:
        hdr = f.read()
    declared = set(re.findall(r"^(?:int|uint64_t|const char\*)\s+(ldb_[a-z_]+)\(", hdr, re.M))
    assert declared >= {"ldb_scan_file_dev", "ldb_scan_file", "ldb_ctx_create"}
    for sym in declared:
        assert hasattr(L, sym), sym
    assert set(N.EXPORTS) == declared
    assert L.ldb_abi_version() == 1
    assert N.status_str(-1) == "invalid crc"


def test_struct_layouts_match_header():
    from lazydb_amd import _native as N
    assert C.sizeof(N.ScanResult) == 32
    assert N.INDEX_TUPLE.itemsize == 16 and N.ENTRY_TUPLE.itemsize == 48
    assert N.INDEX_TUPLE == coracle.INDEX_TUPLE and N.ENTRY_TUPLE == coracle.ENTRY_TUPLE


def _emu():
    so = os.path.join(ROOT, "tests", "emu", "_build", "libldb_emu.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
    L = C.CDLL(so)
    L.emu_scan.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_void_p, C.c_uint64,
                           C.POINTER(coracle.ScanResult), C.c_void_p]
    return L


def emu_scan(img: np.ndarray, io: int):
    L = _emu()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    cap = img.size // 5 + 8
    out = np.zeros(cap, coracle.INDEX_TUPLE)
    res = coracle.ScanResult()
    st = np.zeros(2, np.uint32)
    rc = L.emu_scan(img.ctypes.data if img.size else None, img.size, io, 0, out.ctypes.data, cap, C.byref(res),
                    st.ctypes.data)
    assert rc == 0, rc
    return res, out[: res.n_entries], st


def assert_same(res, tup, ref, rt):
    assert (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries)
    assert np.array_equal(tup["pos"], rt["pos"])
    assert np.array_equal(tup["k_size"], rt["k_size"]) and np.array_equal(tup["v_size"], rt["v_size"])


def test_emulated_engine_golden(golden):
    meta, imgs = golden
    for m in meta:
        img = np.frombuffer(imgs[m["name"]], np.uint8)
        res, tup, st = emu_scan(img, m["io_type"])
        assert (res.status, res.end_off, res.n_entries) == (m["status"], m["end_off"], len(m["tuples"])), m["name"]
        want = [t[0] | (t[1] << 40) | (t[2] << 46) | (t[3] << 52) for t in m["tuples"]]
        assert list(tup["pos"]) == want, m["name"]


@pytest.mark.parametrize("seed", range(4))
def test_emulated_engine_random(seed):
    from tests.golden import make_golden as G
    rng = random.Random(1000 + seed)
    cases = [
        coracle.gen_log(rng.randrange(20000, 300000), seed, ksize=rng.choice([5, 16, 64]),
                        vsize=rng.choice([0, 3, 256, 4000]))[0],
        coracle.gen_log(200000, seed, ksize=64, value_mode=1, zipf_max=512)[0],
        np.frombuffer(G.embedded(seed, 60000), np.uint8).copy(),
        np.frombuffer(G.binary_values(seed, 60000), np.uint8).copy(),
    ]
    for img in cases:
        for _ in range(rng.randrange(0, 3)):
            img[rng.randrange(img.size)] ^= rng.randrange(1, 256)
        for io in (0, 1):
            res, tup, st = emu_scan(img, io)
            ref, rt = coracle.scan(img, io)
            assert_same(res, tup, ref, rt)
