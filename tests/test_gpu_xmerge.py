"""GPU parity of the cross-GPU merge (lazydb_amd/xmerge.py: summary exchange + ldb_merge_files_dev +
ldb_merge_repack_dev), one process playing every rank, against the C oracle's single merge of all
files (db.go:383-427 / 243-265 / 473-523 over the index of index.go:15-26).

Bit-exact: the ranks' streams concatenated in rank order, every ValuePos, the rollover segments
(rank-local runs joined at rank boundaries), the liveness flags, per-file stats and the final
(active fid, append offset)."""
import numpy as np
import pytest

from oracle import coracle
from tests import merge_cases as MC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng(gpu_engine):
    return gpu_engine


def to_dev(img):
    import torch
    return torch.from_numpy(np.ascontiguousarray(img, dtype=np.uint8)).to("cuda:0")


def blocks_of(n_files, world):
    """Contiguous fid blocks, as even as possible, in rank order."""
    b = np.array_split(np.arange(n_files), world)
    return [[int(i) for i in x] for x in b]


def run_ranks(eng, dfiles, world, kw):
    import torch
    from lazydb_amd import xmerge as X
    io = kw.get("io_type", 0)
    blocks = blocks_of(len(dfiles), world)
    max_fid = max(f[1] for f in dfiles)
    own = [[dfiles[i] for i in b] for b in blocks]
    summ = [X.rank_summary(eng, fs, io)[0] for fs in own]
    parts = [X.rank_merge(eng, own[r], summ[r + 1:], X.summary_fid_base(max_fid) + r + 1, kw["active_fid"],
                          kw["active_off"], kw["max_file_size"], kw["now"], io) for r in range(world)]
    sizes = [X.entry_sizes(eng, p) for p in parts]
    places = [X.rank_place(eng, parts[r], torch.cat(sizes[:r]) if r else None, kw["active_fid"], kw["active_off"],
                           kw["max_file_size"]) for r in range(world)]
    return blocks, parts, places


def join(blocks, parts, places):
    stream = np.concatenate([p["stream"].cpu().numpy() for p in parts])
    pos, segs, base = [], [], 0
    for b, p, pl in zip(blocks, parts, places):
        q = pl["pos"].copy()
        q["src_file"] += b[0]
        pos.append(q)
        for sg in pl["segments"]:
            sg = sg.copy()
            sg["stream_off"] += base
            if segs and segs[-1]["fid"] == sg["fid"] and \
                    segs[-1]["file_off"] + segs[-1]["n_bytes"] == sg["file_off"]:
                segs[-1]["n_bytes"] += sg["n_bytes"]
            else:
                segs.append(sg)
        base += int(p["stream"].numel())
    pos = np.concatenate(pos) if pos else np.zeros(0, coracle.MERGE_POS)
    segs = np.array(segs, dtype=coracle.MERGE_SEGMENT) if segs else np.zeros(0, coracle.MERGE_SEGMENT)
    live = np.concatenate([p["live"].cpu().numpy() for p in parts])
    stats = np.concatenate([p["stats"] for p in parts])
    return stream, pos, segs, live, stats


def run_ranks_hashed(engs, dfiles, world, kw):
    """The hash-partitioned merge (xmerge.hashed_sim): route, resolve at the key owners, apply."""
    from lazydb_amd import xmerge as X
    blocks = blocks_of(len(dfiles), world)
    own = [[dfiles[i] for i in b] for b in blocks]
    parts, places = X.hashed_sim(engs[:world], own, kw["active_fid"], kw["active_off"], kw["max_file_size"],
                                 kw["now"], kw.get("io_type", 0))
    return blocks, parts, places


@pytest.fixture(scope="module")
def engs():
    from lazydb_amd import Engine
    es = [Engine(0) for _ in range(8)]
    yield es
    for e in es:
        e.close()


def check(eng, files, kw, world, hashed_engs=None):
    io = kw.get("io_type", 0)
    ref, stream, pos, segs, live, stats = coracle.merge(files, kw["active_fid"], kw["active_off"],
                                                        kw["max_file_size"], kw["now"], io)
    dfiles = [(to_dev(f[0]), f[1], f[2]) for f in files]
    run = (lambda: run_ranks_hashed(hashed_engs, dfiles, world, kw)) if hashed_engs else \
        (lambda: run_ranks(eng, dfiles, world, kw))
    if ref.status != 0:   # a file's replay fails (index.go:90 Fatalf): the rank holding it reports it
        from lazydb_amd import _native as N
        with pytest.raises(N.LdbError):
            run()
        return ref
    blocks, parts, places = run()
    g_stream, g_pos, g_segs, g_live, g_stats = join(blocks, parts, places)
    assert places[-1]["end"] == (ref.end_fid, ref.end_off)
    for r in range(1, world):
        assert places[r]["start"] == places[r - 1]["end"]
    assert len(g_pos) == ref.n_emit and g_pos.tobytes() == pos.tobytes()
    assert g_segs.tobytes() == segs.tobytes()
    assert np.array_equal(g_live, live)
    for k in ("status", "fid", "n_entries", "end_off", "live_count", "live_bytes"):
        assert np.array_equal(g_stats[k], stats[k]), k
    assert int(g_stats["live_count"].sum()) == ref.n_live
    assert g_stream.tobytes() == stream.tobytes()
    return ref


@pytest.mark.parametrize("name", sorted(MC.small_cases()))
def test_xmerge_small_cases(eng, name):
    files, kw = MC.small_cases()[name]
    if len(files) < 2:
        pytest.skip("one file: nothing to split")
    for world in (2, len(files)):
        check(eng, files, kw, world)


@pytest.mark.parametrize("seed,world", [(11, 2), (12, 3), (13, 4)])
def test_xmerge_medium_mixed(eng, seed, world):
    # 4 files x 32 MiB, 2% deletes, 5% expiring records, rollover every 8 MiB: rank pieces cross files
    files, kw = MC.case_generated(seed, n_files=4, cap=32 << 20, n_records=4 * 101_000, max_file_size=8 << 20,
                                  p_delete=20_000, p_expire=50_000, ksize=64, vsize=256)
    ref = check(eng, files, kw, world)
    assert ref.n_emit > 100_000 and ref.n_segments >= 4


def test_xmerge_config5_8_ranks(eng):
    # BASELINE config 5 split as on 8 GPUs: 16 x 256 MiB, half the records stale, 15 targets
    imgs, n, ends = coracle.gen_merge(16, 256 << 20, 16 * 808_540, 3, ksize=64, vsize=256)
    files = [(imgs[i], i + 1, i < 15) for i in range(16)]
    ref = check(eng, files, dict(active_fid=16, active_off=ends[15], max_file_size=256 << 20, now=MC.NOW), 8)
    assert ref.n_live == n // 2


# ---- the hash-partitioned form: ldb_merge_route_dev / resolve / apply


@pytest.mark.parametrize("name", sorted(MC.small_cases()))
def test_xmerge_hashed_small_cases(eng, engs, name):
    files, kw = MC.small_cases()[name]
    for world in sorted({1, 2, min(len(files), 8)}):
        check(eng, files, kw, world, hashed_engs=engs)


@pytest.mark.parametrize("seed,world", [(21, 2), (22, 3), (23, 5), (24, 8)])
def test_xmerge_hashed_medium_mixed(eng, engs, seed, world):
    files, kw = MC.case_generated(seed, n_files=8, cap=16 << 20, n_records=8 * 50_000, max_file_size=8 << 20,
                                  p_delete=20_000, p_expire=50_000, ksize=64, vsize=256)
    ref = check(eng, files, kw, world, hashed_engs=engs)
    assert ref.n_emit > 50_000


def test_xmerge_hashed_config5_8_ranks(eng, engs):
    imgs, n, ends = coracle.gen_merge(16, 256 << 20, 16 * 808_540, 3, ksize=64, vsize=256)
    files = [(imgs[i], i + 1, i < 15) for i in range(16)]
    ref = check(eng, files, dict(active_fid=16, active_off=ends[15], max_file_size=256 << 20, now=MC.NOW), 8,
                hashed_engs=engs)
    assert ref.n_live == n // 2


@pytest.mark.parametrize("world", [1, 2])
def test_xmerge_hashed_all_empty_keys(eng, engs, world):
    """every record has the empty key (str.go accepts nil keys; the golden fixtures hold
    them). The owner of "" receives route records but no key bytes (pad16(0) = 0), which must still
    resolve: last-writer-wins over the one key, an SDelete in between."""
    from tests.merge_cases import _log
    a = _log([dict(key=b"", value=b"v%d" % i) for i in range(5)], 4096)
    b = _log([dict(key=b"", value=b"", stat=1)] + [dict(key=b"", value=b"w%d" % i) for i in range(3)], 4096)
    c = np.zeros(4096, dtype=np.uint8)   # the empty active file
    files = [(a, 1, True), (b, 2, True), (c, 3, False)]
    ref = check(eng, files, dict(active_fid=3, active_off=0, max_file_size=1 << 20, now=MC.NOW), world,
                hashed_engs=engs)
    assert ref.n_live == 1 and ref.n_emit == 1
