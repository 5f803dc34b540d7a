"""GPU parity: liblazydb_gpu.so (called through its C ABI) vs the CPU oracle.

Bit-exact: status, end offset, entry count and every tuple field (offsets, header
sizes, EncodeEntry sizes, stat, key/value sizes; ENTRY kind adds crc, expiredAt,
txid, txstat, fid).
"""
import random
import zlib

import numpy as np
import pytest

from oracle import coracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(gpu_engine):
    return gpu_engine


def to_dev(img):
    import torch
    return torch.from_numpy(np.ascontiguousarray(img, dtype=np.uint8)).to("cuda:0")


def assert_same(res, tup, ref, rt, kind=0):
    assert (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries), \
        (res.as_dict(), (ref.status, ref.end_off, ref.n_entries))
    if kind == 0:
        assert np.array_equal(tup["pos"], rt["pos"])
        assert np.array_equal(tup["k_size"], rt["k_size"]) and np.array_equal(tup["v_size"], rt["v_size"])
    else:
        assert tup.tobytes() == rt.tobytes()


def test_golden_fixtures_device_api(eng, golden):
    meta, imgs = golden
    for m in meta:
        img = np.frombuffer(imgs[m["name"]], np.uint8)
        res, tup = eng.scan_dev(to_dev(img) if img.size else to_dev(np.zeros(0, np.uint8)), io_type=m["io_type"])
        assert (res.status, res.end_off, res.n_entries) == (m["status"], m["end_off"], len(m["tuples"])), m["name"]
        want = [t[0] | (t[1] << 40) | (t[2] << 46) | (t[3] << 52) for t in m["tuples"]]
        assert list(tup["pos"]) == want, m["name"]
        assert list(tup["k_size"]) == [t[4] for t in m["tuples"]], m["name"]


def test_golden_fixtures_host_api_and_entry_kind(eng, golden):
    meta, imgs = golden
    for m in meta:
        img = np.frombuffer(imgs[m["name"]], np.uint8)
        res, tup = eng.scan_host(img, fid=3, io_type=m["io_type"], kind=1)
        ref, rt = coracle.scan(img, m["io_type"], fid=3, tuple_kind=1)
        assert_same(res, tup, ref, rt, kind=1)


def test_serial_walker_matches(eng, golden):
    meta, imgs = golden
    for m in meta[:20]:
        img = np.frombuffer(imgs[m["name"]], np.uint8)
        if img.size == 0:
            continue
        res, tup = eng.scan_dev(to_dev(img), io_type=m["io_type"], serial=True)
        assert (res.status, res.end_off, res.n_entries) == (m["status"], m["end_off"], len(m["tuples"])), m["name"]


@pytest.mark.parametrize("seed", range(8))
def test_random_mutated_logs(eng, seed):
    from tests.golden import make_golden as G
    rng = random.Random(seed)
    cases = [
        coracle.gen_log(rng.randrange(100000, 3 << 20), seed, ksize=rng.choice([5, 16, 64]),
                        vsize=rng.choice([0, 3, 100, 256, 4000]))[0],
        coracle.gen_log(4 << 20, seed + 100, ksize=64, value_mode=1, zipf_max=4096)[0],
        np.frombuffer(G.embedded(seed, 200000), np.uint8).copy(),
        np.frombuffer(G.binary_values(seed, 200000), np.uint8).copy(),
        np.frombuffer(G.mixed(seed, 300000), np.uint8).copy(),
    ]
    for img in cases:
        m = rng.random()
        if m < 0.4:
            for _ in range(rng.randrange(1, 4)):
                img[rng.randrange(img.size)] ^= rng.randrange(1, 256)
        elif m < 0.6:
            img = img[: rng.randrange(img.size)].copy()
        for io in (0, 1):
            res, tup = eng.scan_dev(to_dev(img), io_type=io)
            ref, rt = coracle.scan(img, io)
            assert_same(res, tup, ref, rt)


def test_capacity_reporting(eng):
    img, n, end = coracle.gen_log(1 << 20, 7, ksize=16, vsize=50)
    res, tup = eng.scan_dev(to_dev(img), cap=100)
    assert res.status == -3 and res.n_entries == n and len(tup) == 100
    ref, rt = coracle.scan(img)
    assert np.array_equal(tup["pos"], rt["pos"][:100])


def test_config2_1gib_full_parity(eng):
    """BASELINE config 2: one 1 GiB file of 64-B key / 256-B value entries (FileIO bound)."""
    img, n, end = coracle.gen_log(1 << 30, 1, ksize=64, vsize=256)
    assert n == 3234162 and end == 1073741784
    d = to_dev(img)
    res, tup = eng.scan_dev(d, cap=n + 16)
    ref, rt = coracle.scan(img)
    assert_same(res, tup, ref, rt)
    assert res.status == 2 and res.n_repairs == 0
    # the run prefix (k_uniform) must carry the equal-sized entries, and the chained fast path
    # (ldb_chain.h) the rest: a broken check would only show up here, as the scan silently falling
    # back to the exact general routine
    assert res.n_run == n, (res.n_run, n)
    assert res.n_fast >= 0.9 * res.n_regions, (res.n_fast, res.n_regions)


def test_config3_shape_fast_path(eng):
    """BASELINE config 3 shape (Zipf values 16 B .. 64 KiB) at 256 MiB: parity, and the sweep tier (ldb_sweep.h)
    carrying the whole file (round 5 asserted the region pipeline's fast-region share here, which became
    0 >= 0 once the tier took everything: VERDICT r5 weak #1)."""
    img, n, end = coracle.gen_log(256 << 20, 2, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
    res, tup = eng.scan_dev(to_dev(img), cap=n + 16)
    ref, rt = coracle.scan(img)
    assert_same(res, tup, ref, rt)
    assert res.n_sweep == n and res.n_regions == 0, res.as_dict()


def test_zero_tail_and_zero_values(eng):
    """Preallocated zero tails (config 1 shape, fileio.go:66-68) and zero-valued entries spanning
    regions: the zero-region shortcut of the lean path must give the oracle's tuples exactly."""
    from oracle import pyoracle as P
    img, n, end = coracle.gen_log(64 << 20, 5, ksize=64, vsize=256, max_entries=60_000)
    rng = random.Random(3)
    ents = bytearray()
    for i in range(3000):
        vl = rng.choice([0, 100, 7000, 12000, 16000])
        ents += P.encode_entry(P.Entry(key=b"zk%05d" % i, value=bytes(vl), k_size=6, v_size=vl))
    zeroval = np.frombuffer(bytes(ents) + bytes(1 << 20), np.uint8).copy()
    for im in (img, zeroval):
        for io in (0, 1):
            res, tup = eng.scan_dev(to_dev(im), io_type=io)
            ref, rt = coracle.scan(im, io)
            assert_same(res, tup, ref, rt)
            if im is img:   # zeroval has entries under 84 B, which the lean path leaves to region_process
                assert res.n_fast == res.n_regions


def test_config4_4gib_64bit_offsets(eng):
    """BASELINE config 4's per-GPU file shape (64/256 entries, seed 10) at 4.5 GiB, so entry offsets
    pass 2^32 (a 4 GiB file ends 160 B short of it). Full tuple parity, then one corrupted value
    byte beyond 2^32: the scan must stop with
    ErrInvalidCrc at that entry's 64-bit offset, with every earlier tuple delivered
    (log_file.go:141-143, index.go:90)."""
    img, n, end = coracle.gen_log(9 << 29, 10, ksize=64, vsize=256)
    assert n == (9 << 29) // 332 and end > (1 << 32)
    d = to_dev(img)
    res, tup = eng.scan_dev(d, cap=n + 16)
    ref, rt = coracle.scan(img)
    assert_same(res, tup, ref, rt)
    assert res.status == 2 and res.n_repairs == 0
    offs = rt["pos"] & ((1 << 40) - 1)                         # pos bits [0, 40): offset
    k = int(np.searchsorted(offs, (1 << 32) + 12345))          # first entry starting past the mark
    bad = int(offs[k]) + 100
    del tup, rt, offs
    img[bad] ^= 0x5A
    d[bad] = int(img[bad])
    res, tup = eng.scan_dev(d, cap=n + 16)
    ref, rt = coracle.scan(img)
    assert_same(res, tup, ref, rt)
    assert ref.status == -1 and ref.end_off > (1 << 32) and res.n_entries == k


def test_config3_8gib_full_parity(eng):
    """BASELINE config 3 at its full size: one 8 GiB log file (bound 2^33), 64-B keys, values of
    16 * Zipf(1.1, [1, 4096]) bytes (16 B .. 64 KiB; vSize varints of 1-3 bytes). Entry offsets need 34
    bits (they run to within 64 KiB of the 2^33 bound); every tuple, the stop status and the append offset must be the oracle's."""
    img, n, end = coracle.gen_log(8 << 30, 2, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
    assert end > (1 << 33) - (64 << 10)
    d = to_dev(img)
    res, tup = eng.scan_dev(d, cap=n + 16)
    del d
    ref, rt = coracle.scan(img)
    assert_same(res, tup, ref, rt)
    assert ref.n_entries == n and int(rt["pos"][-1] & ((1 << 40) - 1)) > (1 << 33) - (128 << 10)
    assert res.status == 2 and res.n_repairs == 0
    assert res.n_sweep == n, res.as_dict()   # the sweep tier takes the whole file (no silent fallback)


def _fixed_log(n, klen, vlen, seed, expired_at=0, tx_id=0):
    from oracle import pyoracle as P
    rng = random.Random(seed)
    out = bytearray()
    for i in range(n):
        out += P.encode_entry(P.Entry(key=bytes(rng.randrange(97, 123) for _ in range(klen)),
                                      value=bytes(rng.randrange(48, 58) for _ in range(vlen)), k_size=klen,
                                      v_size=vlen, expired_at=expired_at, tx_id=tx_id))
    return bytes(out)


@pytest.mark.parametrize("shape", [(64, 256, 0, 0), (16, 100, 0, 0), (13, 70, 0, 0), (20, 33, 1700000000, 7),
                                   (9, 9, 0, 0), (64, 256, 0, 1 << 40), (16, 361, 0, 0), (40, 1000, 0, 0),
                                   (16, 3041, 0, 0), (64, 5000, 0, 0), (16, 362, 0, 0),
                                   (1, 0, 0, 0), (0, 0, 0, 0), (0, 1, 0, 0), (2, 3, 0, 0), (1, 4, 0, 0)])
def test_run_prefix_shapes(eng, shape):
    """The run prefix (k_uniform): equal-sized entries at the file start (10-B entries up: a header and
    no key or value), then the
    region pipeline from the first entry outside the run. Every span length mod 8, long headers,
    clean and cut ends, corrupted entries at the run's start / middle / end, a run followed by
    other entries; both IOController rules and both tuple kinds (k_uniform writes ldb_entry too)."""
    klen, vlen, exp, txid = shape
    rng = random.Random(klen * 7 + vlen)
    n = 3000 if vlen < 1000 else 600
    run = _fixed_log(n, klen, vlen, rng.randrange(1 << 30), expired_at=exp, tx_id=txid)
    esz = len(run) // n
    other = coracle.gen_log(200_000, 6, ksize=16, vsize=40)
    for tail in (b"", bytes(37), bytes(9000), bytes(other[0][: other[2]]) + bytes(300)):
        base = np.frombuffer(run + tail, np.uint8).copy()
        variants = [base, base[: (n // 2) * esz + 3].copy(), base[: (n - 1) * esz + 30].copy()]
        for k in (0, 1, n // 4, n - 1):
            im = base.copy()
            im[k * esz + rng.choice([0, 5, esz - 1])] ^= 0x40
            variants.append(im)
        for im in variants:
            d = to_dev(im)
            for io in (0, 1):
                for kind in (0, 1):
                    res, tup = eng.scan_dev(d, io_type=io, kind=kind)
                    ref, rt = coracle.scan(im, io, tuple_kind=kind)
                    assert_same(res, tup, ref, rt, kind=kind)


def test_run_prefix_capacity(eng):
    """Fewer output slots than run entries: LDB_ERR_CAPACITY with the full count, the first cap
    tuples exact."""
    img, n, end = coracle.gen_log(4 << 20, 9, ksize=64, vsize=256)
    res, tup = eng.scan_dev(to_dev(img), cap=1000)
    ref, rt = coracle.scan(img)
    assert res.status == -3 and res.n_entries == n and res.n_run == n
    assert np.array_equal(tup["pos"], rt["pos"][:1000])


def _runs_log(spec, seed):
    """Runs of equal-sized entries one after another: spec = [(n, klen, vlen, expired_at), ...]."""
    return b"".join(_fixed_log(n, k, v, seed + 31 * i, expired_at=e) for i, (n, k, v, e) in enumerate(spec))


@pytest.mark.parametrize("case", ["steps", "aligned", "many", "single_between", "repeat", "cut"])
def test_piecewise_runs(eng, case):
    """Round 4: a log that is several runs of equal-sized entries (the reference bench's keys grow a
    digit at entries 10, 100, ...; fixed-schema writers whose key or value width steps) is verified run
    by run in k_uniform: K counts entries along the chain over the runs, x0 follows the runs, and a file
    the runs cover to its terminal needs no region kernel. Runs of every slicing (entries 29 B .. 5 KB,
    starts not dword-aligned), more runs than k_uniform keeps (8; the rest go to the region pipeline), a
    lone entry between runs, a run shape that recurs after another one (the boundary search is then only
    an upper bound), corruption at a run's first, middle and last entry, a 240 KiB zero tail and a cut
    end; both IOController rules, both tuple kinds, bit-exact."""
    rng = random.Random(zlib.crc32(case.encode()))
    if case == "steps":       # the reference bench's shape, small: key widths 16..21
        spec = [(10, 16, 512, 0), (90, 17, 512, 0), (900, 18, 512, 0), (2000, 19, 512, 0), (500, 20, 512, 0)]
    elif case == "aligned":   # 332-B and 100-B entries: dword-aligned runs, and runs whose start is not
        spec = [(700, 64, 256, 0), (333, 13, 75, 0), (701, 64, 256, 0), (50, 9, 9, 0), (300, 40, 1000, 0)]
    elif case == "many":      # 11 runs: k_uniform takes 8
        spec = [(40 + 7 * i, 10 + i, 30 + 13 * i, 0) for i in range(11)]
    elif case == "single_between":   # run, one entry, run (the lone entry is not a run start)
        spec = [(500, 16, 100, 0), (1, 16, 37, 0), (600, 16, 100, 0), (400, 20, 5000, 0)]
    elif case == "repeat":    # A, B, A, B with A and B of equal size (expiry differs): non-monotone headers
        spec = [(300, 16, 100, 0), (200, 16, 100, 1700000000), (300, 16, 100, 0), (200, 16, 100, 1700000001)]
    else:                     # cut inside the last run
        spec = [(100, 16, 200, 0), (1000, 18, 200, 0)]
    log = _runs_log(spec, rng.randrange(1 << 30))
    n_all = sum(x[0] for x in spec)
    bounds = [0]
    for (nn, k, v, e) in spec:
        bounds.append(bounds[-1] + len(_fixed_log(1, k, v, 1, expired_at=e)) * nn)
    imgs = [np.frombuffer(log + bytes(240 << 10), np.uint8).copy()]
    if case == "cut":
        imgs = [np.frombuffer(log[: len(log) - 150], np.uint8).copy()]
    base = imgs[0]
    # corrupt a byte of run 2's (or the last run's) first, middle and last entry
    r = min(2, len(spec) - 1)
    esz = (bounds[r + 1] - bounds[r]) // spec[r][0]
    for k in (0, spec[r][0] // 2, spec[r][0] - 1):
        im = base.copy()
        im[bounds[r] + k * esz + rng.choice([0, 6, esz - 1])] ^= 0x20
        imgs.append(im)
    for i, im in enumerate(imgs):
        d = to_dev(im)
        for io in (0, 1):
            for kind in (0, 1):
                res, tup = eng.scan_dev(d, io_type=io, kind=kind, cap=n_all + 64)
                ref, rt = coracle.scan(im, io, tuple_kind=kind, cap=n_all + 64)
                assert_same(res, tup, ref, rt, kind=kind)
                if i == 0 and case in ("steps", "aligned") and kind == 0:
                    # every run went through k_uniform and it ended the scan (no region kernel)
                    assert res.n_run == n_all and res.n_regions == 0, (res.n_run, n_all, res.n_regions)


@pytest.mark.parametrize("io_type", [1, 0])
def test_config1_reference_bench_log(eng, io_type):
    """BASELINE config 1 at its stated size, in the reference benchmark's own shape
    (bench/db_bench_test.go:17-36, :63-68): 500 K Sets of "bench_test_key_<i>" (16..21-B keys, so the
    entry size changes at i = 10, 100, ..., 100000) with 512-B alphabet values, in one 512 MiB
    preallocated file, scanned under the Mmap rule (IOType = 1: o + n >= len is EOF,
    iocontroller/mmap.go:46-52) and under FileIO. Both tuple kinds, bit-exact."""
    img, n, end = coracle.gen_bench_log(512 << 20, 11, n_entries=500_000)
    assert n == 500_000 and end == 271_888_890
    d = to_dev(img)
    ref, rt = coracle.scan(img, io_type)
    assert ref.status == 2 and ref.end_off == end and ref.n_entries == n
    res, tup = eng.scan_dev(d, io_type=io_type, cap=n + 16)
    assert_same(res, tup, ref, rt)
    # round 4: its six runs (key widths 16..21) all go through k_uniform, which ends the scan at the
    # sentinel, so the 240 MiB zero tail is never staged
    assert res.n_run == n and res.n_regions == 0, (res.n_run, res.n_regions)
    res1, tup1 = eng.scan_dev(d, io_type=io_type, cap=n + 16, kind=1)
    ref1, rt1 = coracle.scan(img, io_type, tuple_kind=1)
    assert_same(res1, tup1, ref1, rt1, kind=1)


@pytest.mark.parametrize("io_type", [0, 1])
def test_writer_realistic_mix(eng, io_type):
    """What LazyDB's writers append, interleaved (str.go Set/SetEX/Delete, tx.go Commit): 64 MiB,
    bit-exact under both IO rules, and with the file truncated mid-entry (EOF_KV / EOF_WINDOW)."""
    img, n, end = coracle.gen_writer_log(64 << 20, 21)
    d = to_dev(img)
    res, tup = eng.scan_dev(d, io_type=io_type, cap=n + 16)
    ref, rt = coracle.scan(img, io_type)
    assert_same(res, tup, ref, rt)
    assert res.n_entries == n
    assert res.n_sweep >= 0.95 * n, res.as_dict()   # the sweep tier carries it
    for cut in (end - 7, end - 300, end // 2 + 13):
        part = np.ascontiguousarray(img[:cut])
        res, tup = eng.scan_dev(to_dev(part), io_type=io_type, cap=n + 16)
        ref, rt = coracle.scan(part, io_type)
        assert_same(res, tup, ref, rt)
