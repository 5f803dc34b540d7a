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
    assert L.ldb_abi_version() == 4
    assert N.status_str(-1) == "invalid crc"


def test_struct_layouts_match_header():
    from lazydb_amd import _native as N
    assert C.sizeof(N.ScanResult) == 56
    assert N.INDEX_TUPLE.itemsize == 16 and N.ENTRY_TUPLE.itemsize == 48
    assert N.INDEX_TUPLE == coracle.INDEX_TUPLE and N.ENTRY_TUPLE == coracle.ENTRY_TUPLE


def _emu():
    so = os.path.join(ROOT, "tests", "emu", "_build", "libldb_emu.so")
    if not os.path.exists(so):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "emu")], check=True)
    L = C.CDLL(so)
    L.emu_scan_runs.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_void_p, C.c_uint64,
                                C.POINTER(coracle.ScanResult), C.c_void_p, C.c_uint64]
    return L


# regions per wavefront run: 0 = every region speculative (region_process only); >0 = contiguous
# runs through the chained fast path (ldb_chain.h), as k_scan_main assigns them
RUNS = [0, 1, 3, 64]


def emu_scan(img: np.ndarray, io: int, run_len: int = 0):
    L = _emu()
    img = np.ascontiguousarray(img, dtype=np.uint8)
    cap = img.size // 5 + 8
    out = np.zeros(cap, coracle.INDEX_TUPLE)
    res = coracle.ScanResult()
    st = np.zeros(4, np.uint32)
    rc = L.emu_scan_runs(img.ctypes.data if img.size else None, img.size, io, 0, out.ctypes.data, cap, C.byref(res),
                         st.ctypes.data, run_len)
    assert rc == 0, rc
    return res, out[: res.n_entries], st


def assert_same(res, tup, ref, rt):
    assert (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries)
    assert np.array_equal(tup["pos"], rt["pos"])
    assert np.array_equal(tup["k_size"], rt["k_size"]) and np.array_equal(tup["v_size"], rt["v_size"])


@pytest.mark.parametrize("run_len", RUNS)
def test_emulated_engine_golden(golden, run_len):
    meta, imgs = golden
    for m in meta:
        img = np.frombuffer(imgs[m["name"]], np.uint8)
        res, tup, st = emu_scan(img, m["io_type"], run_len)
        assert (res.status, res.end_off, res.n_entries) == (m["status"], m["end_off"], len(m["tuples"])), m["name"]
        want = [t[0] | (t[1] << 40) | (t[2] << 46) | (t[3] << 52) for t in m["tuples"]]
        assert list(tup["pos"]) == want, m["name"]


@pytest.mark.parametrize("run_len", RUNS)
@pytest.mark.parametrize("seed", range(4))
def test_emulated_engine_random(seed, run_len):
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
            res, tup, st = emu_scan(img, io, run_len)
            ref, rt = coracle.scan(img, io)
            assert_same(res, tup, ref, rt)


@pytest.mark.parametrize("walkers", ["0", "rev", "fwd"])
def test_emulated_two_phase_repair(golden, walkers, monkeypatch):
    """k_repair's two phases (ldb_pipeline.h walk_source, then the links again and the serial
    repair): the result is the oracle's whatever the walkers did -- none ("0", the serial repair
    alone), in flag order, or in reverse flag order, where every walker starts from a source an
    earlier walker has yet to rewrite and loses claims to it. Adversarial logs (values holding valid
    entries, every header field varied, random binary) break links in most regions."""
    from tests.golden import make_golden as G
    monkeypatch.setenv("LDB_EMU_WALKERS", walkers)
    meta, imgs = golden
    cases = [np.frombuffer(imgs[m["name"]], np.uint8) for m in meta]
    for seed in range(2):
        for gen in (G.embedded, G.mixed, G.binary_values):
            b = np.frombuffer(gen(50 + seed, 150000), np.uint8)
            ref, _ = coracle.scan(b)
            cases.append(np.concatenate([np.tile(b[: ref.end_off], 3), np.zeros(64, np.uint8)]))
    for img in cases:
        for io in (0, 1):
            for run_len in (0, 1, 3):
                res, tup, st = emu_scan(img, io, run_len)
                ref, rt = coracle.scan(img, io)
                assert_same(res, tup, ref, rt)


def _log_with_entry_at(target: int, big_value: int, seed: int) -> np.ndarray:
    """Entries of 16-B keys and 100-B values (128-B entries) up to `target`, one 12-B-header
    filler that makes the next entry start exactly at `target`, that entry with a `big_value`-byte
    value, then a short tail entry."""
    from oracle import pyoracle as P
    rng = random.Random(seed)
    out = bytearray()

    def ent(klen, vlen):
        return P.encode_entry(P.Entry(key=bytes(rng.randrange(97, 123) for _ in range(klen)),
                                      value=bytes(rng.randrange(48, 58) for _ in range(vlen)), k_size=klen,
                                      v_size=vlen))
    while target - len(out) > 128 + 200:
        out += ent(16, 100)
    gap = target - len(out) - 10          # header of (k=0 or small, v) is 10 B while v < 64
    klen = 8
    vlen = gap - klen
    if vlen >= 64:                        # 2-byte vsize varint: one byte less of value
        vlen -= 1
    e = ent(klen, vlen)
    assert len(out) + len(e) == target, (len(out), len(e), target)
    out += e
    out += ent(16, big_value)
    out += ent(16, 40)
    return np.frombuffer(bytes(out) + bytes(64), np.uint8).copy()


@pytest.mark.parametrize("run_len", [0, 64])
@pytest.mark.parametrize("d", [-9, -8, -7, -5, -4, -3, -2, -1, 0, 1])
@pytest.mark.parametrize("big", [200, 6000, 12000])
def test_emulated_span_starting_at_region_boundary(d, big, run_len):
    """The entry's CRC span (offset+4) starts d+4 bytes after region 1's start (d = -4..-1: the
    stored crc straddles the boundary; the k_combine skip path) and ends in the next region, a
    covered region later, or two regions later; both intact and with a flipped byte."""
    R1 = 5120
    img = _log_with_entry_at(R1 + d, big, seed=d * 31 + big)
    for flip in (None, R1 + d + 4 + big // 2, R1 + d + 2):
        im = img.copy()
        if flip is not None:
            im[flip] ^= 0x20
        for io in (0, 1):
            res, tup, st = emu_scan(im, io, run_len)
            ref, rt = coracle.scan(im, io)
            assert_same(res, tup, ref, rt)


@pytest.mark.parametrize("seed", range(3))
def test_emulated_chained_path(seed):
    """Contiguous runs through the chained fast path (ldb_chain.h): entry sizes 93 B .. ~1.1 KiB
    put entry starts (and their stored-crc fields) at every offset of a slice, including the last
    4 bytes (owner checked by the next lane) and the last 8 bytes of a region (fallback). Intact
    logs must take the fast path for most regions; single-byte corruptions anywhere (headers,
    crc fields, values) must give exactly the oracle's result."""
    img, n, end = coracle.gen_log(600_000, 40 + seed, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=64)
    nreg = (img.size + 5119) // 5120
    res, tup, st = emu_scan(img, 0, 64)
    ref, rt = coracle.scan(img, 0)
    assert_same(res, tup, ref, rt)
    assert st[2] >= 0.8 * nreg, (int(st[2]), nreg)      # regions done by the fast path
    rng = random.Random(seed)
    for _ in range(12):
        im = img.copy()
        at = rng.randrange(0, end)
        im[at] ^= 1 << rng.randrange(8)
        for io in (0, 1):
            res, tup, st = emu_scan(im, io, 64)
            ref, rt = coracle.scan(im, io)
            assert_same(res, tup, ref, rt)


@pytest.mark.parametrize("seed", range(3))
def test_emulated_file_end(seed):
    """End of file on the chained fast path (ldb_chain.h lean_terminal / covered tail region): logs
    cut at many lengths (inside entries: EOF_KV, window EOF, CRC errors once zero padding follows)
    and clean ends (exactly at the last entry, or zero padding: EOF_WINDOW / sentinel / a covered
    zero tail region), both IOController bound rules; every result must be the oracle's, and clean
    ends must stay on the fast path for every region (except the mmap rule's EOF_KV on an entry
    that ends exactly at the file end, log_file.go:130-139, which region_process reports)."""
    base, n, end = coracle.gen_log(60_000 + 1000 * seed, 7 + seed, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=64)
    rng = random.Random(seed)
    for cut in [rng.randrange(end - 400, end) for _ in range(6)] + [rng.randrange(5000, end) for _ in range(4)]:
        for pad in (0, 10, 38, 200):
            img = np.concatenate([base[:cut], np.zeros(pad, np.uint8)])
            for io in (0, 1):
                res, tup, st = emu_scan(img, io, 64)
                ref, rt = coracle.scan(img, io)
                assert_same(res, tup, ref, rt)
    for pad in (0, 10, 37, 38, 40, 64, 4000):
        img = np.concatenate([base[:end], np.zeros(pad, np.uint8)])
        nreg = (img.size + 5119) // 5120
        for io in (0, 1):
            res, tup, st = emu_scan(img, io, 64)
            ref, rt = coracle.scan(img, io)
            assert_same(res, tup, ref, rt)
            if not (pad == 0 and io == 1):
                assert int(st[2]) == nreg, (pad, io, int(st[2]), nreg)


@pytest.mark.parametrize("run_len", [1, 3, 64])
def test_emulated_zero_regions(run_len):
    """All-zero regions (the preallocated tail of a log file, fileio.go:66-68; zero-valued entries)
    take the zero-region shortcut of the speculative lean path (ldb_chain.h): a zero tail after the
    last entry, zero tails followed by garbage, and chains running through zero-valued entries that
    span whole regions, with runs starting inside the zeros; intact and with flipped bytes."""
    from oracle import pyoracle as P
    rng = random.Random(5 + run_len)
    base, n, end = coracle.gen_log(40_000, 3, ksize=64, vsize=256)
    tail = np.concatenate([base[:end], np.zeros(60_000, np.uint8)])
    garbage = tail.copy()
    garbage[-3000:] = np.frombuffer(bytes(rng.randrange(256) for _ in range(3000)), np.uint8)
    ents = bytearray()
    for i in range(12):
        vl = rng.choice([0, 100, 7000, 12000, 16000])
        ents += P.encode_entry(P.Entry(key=b"zk%03d" % i, value=bytes(vl), k_size=5, v_size=vl))
    zeroval = np.frombuffer(bytes(ents) + bytes(20_000), np.uint8).copy()
    for img in (tail, garbage, zeroval):
        nreg = (img.size + 5119) // 5120
        for flip in (None, rng.randrange(img.size // 2)):
            im = img.copy()
            if flip is not None:
                im[flip] ^= 0x04
            for io in (0, 1):
                res, tup, st = emu_scan(im, io, run_len)
                ref, rt = coracle.scan(im, io)
                assert_same(res, tup, ref, rt)
                if flip is None and img is tail:
                    assert int(st[2]) == nreg


@pytest.mark.parametrize("seed", range(4))
def test_emulated_predicted_starts(seed):
    """Chained regions of equal-sized entries take the predicted-start route (ChainState memo,
    ldb_chain.h predict_starts): every chain position is verified by a header-byte compare. Logs
    whose entry size changes mid-run, corrupted headers (a size varint, the Status byte, a zeroed crc
    field), corrupted values and cut ends must all give exactly the oracle's result."""
    from oracle import pyoracle as P
    rng = random.Random(70 + seed)
    a = coracle.gen_log(300_000, 80 + seed, ksize=64, vsize=256)
    b = coracle.gen_log(200_000, 90 + seed, ksize=16, vsize=100)
    c = coracle.gen_log(150_000, 95 + seed, ksize=64, vsize=256)
    # three runs of different entry sizes back to back, then the zero tail of a preallocated file
    img = np.concatenate([a[0][: a[2]], b[0][: b[2]], c[0][: c[2]], np.zeros(9000, np.uint8)])
    ends = [0, a[2], a[2] + b[2], a[2] + b[2] + c[2]]
    res, tup, st = emu_scan(img, 0, 64)
    ref, rt = coracle.scan(img, 0)
    assert_same(res, tup, ref, rt)
    starts = rt["pos"] & ((1 << 40) - 1)
    for trial in range(14):
        im = img.copy()
        kind = trial % 7
        k = rng.randrange(1, len(starts) - 1)
        s0 = int(starts[k])
        if kind == 0:
            im[s0 + 10] ^= 0x02          # a size varint byte: the header no longer equals the memo
        elif kind == 1:
            im[s0 + 4] = 1               # Status SDelete: a different (valid-looking) header
        elif kind == 2:
            im[s0: s0 + 4] = 0           # zeroed crc field at a predicted start
        elif kind == 3:
            im[s0 + 40] ^= 0x10          # a value byte: the owner check fails
        elif kind == 4:
            im = im[: s0 + rng.randrange(1, 300)].copy()   # cut inside an entry
        elif kind == 5:
            im = np.concatenate([im[: ends[rng.randrange(1, 4)]], np.zeros(rng.choice([0, 10, 38, 5000]), np.uint8)])
        else:
            e = P.encode_entry(P.Entry(key=b"k" * 64, value=b"v" * 256, k_size=64, v_size=256, expired_at=5))
            im[s0: s0 + len(e)] = np.frombuffer(e, np.uint8)   # a valid entry of another header shape
        for io in (0, 1):
            res, tup, st = emu_scan(im, io, 64)
            ref, rt = coracle.scan(im, io)
            assert_same(res, tup, ref, rt)


def emu_scan_run(img: np.ndarray, io: int, run_len: int = 64):
    """The emulated pipeline with the run prefix (k_uniform) first."""
    L = _emu()
    if not hasattr(L.emu_scan_ex, "_typed"):
        L.emu_scan_ex.argtypes = [C.c_void_p, C.c_uint64, C.c_int, C.c_uint32, C.c_void_p, C.c_uint64,
                                  C.POINTER(coracle.ScanResult), C.c_void_p, C.c_uint64, C.c_int]
        L.emu_scan_ex._typed = True
    img = np.ascontiguousarray(img, dtype=np.uint8)
    cap = img.size // 5 + 8
    out = np.zeros(cap, coracle.INDEX_TUPLE)
    res = coracle.ScanResult()
    st = np.zeros(4, np.uint32)
    rc = L.emu_scan_ex(img.ctypes.data if img.size else None, img.size, io, 0, out.ctypes.data, cap, C.byref(res),
                       st.ctypes.data, run_len, 1)
    assert rc == 0, rc
    return res, out[: res.n_entries], st


def _fixed_log(n, klen, vlen, seed, expired_at=0, tx_id=0, stat=0):
    from oracle import pyoracle as P
    rng = random.Random(seed)
    out = bytearray()
    for i in range(n):
        out += P.encode_entry(P.Entry(key=bytes(rng.randrange(97, 123) for _ in range(klen)),
                                      value=bytes(rng.randrange(48, 58) for _ in range(vlen)), k_size=klen,
                                      v_size=vlen, expired_at=expired_at, tx_id=tx_id, stat=stat))
    return out


@pytest.mark.parametrize("shape", [(64, 256, 0, 0), (16, 100, 0, 0), (13, 70, 0, 0), (20, 33, 1700000000, 7),
                                   (9, 9, 0, 0), (5, 0, 0, 0), (64, 256, 0, 1 << 40)])
def test_emulated_run_prefix(shape):
    """The run prefix (k_uniform, ldb_pipeline.h uni_*): equal-sized entries at the file start are
    verified one per lane, and the region pipeline resumes at the first entry outside the run. Entry
    sizes with every span length mod 8, long headers (a 5-byte ExpiredAt), a 6-byte TxID, tiny
    entries; clean ends (exact, zero tail, short tail), corrupted entries at the run's start, middle
    and end, a run followed by entries of another size, and both IOController rules."""
    klen, vlen, exp, txid = shape
    rng = random.Random(klen * 1000 + vlen)
    run = _fixed_log(300, klen, vlen, rng.randrange(1 << 30), expired_at=exp, tx_id=txid)
    esz = len(run) // 300
    other = coracle.gen_log(40_000, 5, ksize=16, vsize=40)
    tails = [b"", bytes(10), bytes(37), bytes(38), bytes(9000), bytes(other[0][: other[2]]) + bytes(300)]
    for tail in tails:
        base = np.frombuffer(bytes(run) + tail, np.uint8).copy()
        variants = [base]
        for k in (0, 150, 299):
            for off in (0, 5, esz - 1):
                im = base.copy()
                im[k * esz + off] ^= 0x40
                variants.append(im)
        variants.append(base[: 150 * esz + 3].copy())
        variants.append(base[: 299 * esz + 30].copy())
        for im in variants:
            for io in (0, 1):
                res, tup, st = emu_scan_run(im, io)
                ref, rt = coracle.scan(im, io)
                assert_same(res, tup, ref, rt)


# value lengths whose CRC spans (L = sz - 4, header 10 B for these keys) land on every slicing of
# uni_geometry: G = 1..64 lanes per entry, span lengths at each G's bounds, leads longer than a window
# (t > P: whole windows masked), and just past the largest run size (no run)
_GEOM_VLENS = [0, 1, 7, 8, 30, 31, 32, 33, 34, 90, 91, 120, 121, 122, 300, 310, 311, 312, 313, 315, 330, 361, 362, 363, 400, 700,
               760, 761, 1000, 1500, 1520, 1521, 2900, 3000, 3040, 3041, 4000, 6000, 6090, 6091, 6092, 7000]


def test_emulated_run_geometries():
    """The run prefix's entry-aligned slices (uni_geometry, uni_lead, the group's tree combine) over
    span lengths that exercise every lanes-per-entry count and the masked-lead cases; a clean run is
    covered whole, a corrupted member ends it, and the pipeline agrees with the oracle throughout."""
    for vlen in _GEOM_VLENS:
        rng = random.Random(vlen)
        n = 120 if vlen < 2000 else 40
        run = _fixed_log(n, 16, vlen, rng.randrange(1 << 30))
        esz = len(run) // n
        base = np.frombuffer(bytes(run), np.uint8).copy()
        bad = base.copy()
        bad[(n // 2) * esz + rng.randrange(4, esz)] ^= 0x08
        for im, k in ((base, n), (bad, n // 2)):
            res, tup, st = emu_scan_run(im, 0)
            ref, rt = coracle.scan(im, 0)
            assert_same(res, tup, ref, rt)
            # a member needs its whole header window readable (kMaxHeader bytes, log_file.go:117-122)
            want = min(k, ref.n_entries) if esz - 4 <= 6144 else 0
            assert res.n_run == want, (vlen, esz, res.n_run, want)


def test_emulated_run_prefix_counts():
    """A clean config-2-shaped log is covered by the run: every entry but none of the regions."""
    img, n, end = coracle.gen_log(1 << 20, 3, ksize=64, vsize=256)
    res, tup, st = emu_scan_run(img, 0)
    ref, rt = coracle.scan(img, 0)
    assert_same(res, tup, ref, rt)
    assert res.n_run == n and res.n_regions <= 1
    zipf = coracle.gen_log(1 << 20, 3, ksize=64, value_mode=1, zipf_max=512)[0]
    res, tup, st = emu_scan_run(zipf, 0)
    ref, rt = coracle.scan(zipf, 0)
    assert_same(res, tup, ref, rt)
    assert res.n_run < 50
