"""GPU parity of the merge/GC engine (ldb_merge_files_dev, called through the C ABI) against the C
oracle's restatement of db.go:383-427 / 243-265 / 473-523 over the index of index.go:15-26.

Bit-exact: the compacted stream bytes, every new ValuePos (fid, offset, entry size, source), the
rollover segments, the per-record liveness flags, per-file live counts/bytes and the final
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


def check_case(eng, files, kw):
    io = kw.get("io_type", 0)
    ref, stream, pos, segs, live, stats = coracle.merge(files, kw["active_fid"], kw["active_off"],
                                                        kw["max_file_size"], kw["now"], io)
    dfiles = [(to_dev(f[0]), f[1], f[2]) for f in files]
    out = eng.merge_dev(dfiles, kw["active_fid"], kw["active_off"], kw["max_file_size"], kw["now"], io_type=io)
    r = out["result"]
    assert (r.status, r.bad_file) == (ref.status, ref.bad_file), (r.as_dict(), ref.status, ref.bad_file)
    if ref.status != 0:
        return r
    assert (r.n_records, r.n_live, r.n_emit, r.emit_bytes, r.end_fid, r.end_off, r.n_segments) == \
        (ref.n_records, ref.n_live, ref.n_emit, ref.emit_bytes, ref.end_fid, ref.end_off, ref.n_segments)
    assert out["segments"].tobytes() == segs.tobytes()
    assert out["pos"].tobytes() == pos.tobytes()
    st = out["stats"]
    for k in ("status", "fid", "n_entries", "end_off", "live_count", "live_bytes"):
        assert np.array_equal(st[k], stats[k]), k
    assert np.array_equal(out["live"].cpu().numpy(), live)
    if r.emit_bytes <= (64 << 20):
        assert out["stream"].cpu().numpy().tobytes() == stream.tobytes()
    else:
        import torch
        assert torch.equal(out["stream"], to_dev(stream))
    return r


@pytest.mark.parametrize("name", sorted(MC.small_cases()))
def test_merge_small_cases(eng, name):
    files, kw = MC.small_cases()[name]
    check_case(eng, files, kw)


@pytest.mark.parametrize("name", sorted(MC.small_cases()))
def test_merge_small_cases_tagless(eng, name, monkeypatch):
    """The same cases with the liveness table's hash tag off (LDB_MERGE_TAGLESS): every probe that
    meets a taken slot compares the keys, so the key-length recovery from the bytes before a
    slot's key (key_len_before) and the byte compare decide every duplicate."""
    monkeypatch.setenv("LDB_DEBUG", "1")   # (the library reads its switches only under LDB_DEBUG)
    monkeypatch.setenv("LDB_MERGE_TAGLESS", "1")
    files, kw = MC.small_cases()[name]
    check_case(eng, files, kw)


@pytest.mark.parametrize("seed", [11, 12])
def test_merge_medium_mixed(eng, seed):
    # 4 files x 32 MiB, 64/256 entries, 2% deletes, 5% expiring records, rollover every 8 MiB
    files, kw = MC.case_generated(seed, n_files=4, cap=32 << 20, n_records=4 * 101_000, max_file_size=8 << 20,
                                  p_delete=20_000, p_expire=50_000, ksize=64, vsize=256)
    r = check_case(eng, files, kw)
    assert r.n_emit > 100_000 and r.n_segments >= 4


def test_merge_config5_full(eng):
    # BASELINE config 5: 16 files x 256 MiB, 64/256 entries, exactly half the records stale; 15 targets
    imgs, n, ends = coracle.gen_merge(16, 256 << 20, 16 * 808_540, 3, ksize=64, vsize=256)
    assert n == 16 * 808_540
    files = [(imgs[i], i + 1, i < 15) for i in range(16)]
    r = check_case(eng, files, dict(active_fid=16, active_off=ends[15], max_file_size=256 << 20, now=MC.NOW))
    assert r.n_live == n // 2
