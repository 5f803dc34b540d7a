"""Merge/GC oracle: the C restatement (oracle/ldb_oracle.c ldbo_merge) against the independent Python
twin (oracle/pyoracle.py merge) and against the reference's own pinned rollover positions
(db_test.go:182-229). Parity of the merge output itself is otherwise unpinned in the reference
(db_test.go:64-109 asserts no error only); see DESIGN.md."""
import numpy as np
import pytest

from oracle import coracle
from oracle import pyoracle as P
from tests import merge_cases as MC

CASES = MC.small_cases()


def run_c(files, kw):
    return coracle.merge(files, kw["active_fid"], kw["active_off"], kw["max_file_size"], kw["now"],
                         kw.get("io_type", 0))


@pytest.mark.parametrize("name", sorted(CASES))
def test_c_oracle_matches_python_twin(name):
    files, kw = CASES[name]
    res, stream, pos, segs, live, stats = run_c(files, kw)
    py = P.merge([(f[0].tobytes(), f[1], f[2]) for f in files], kw["active_fid"], kw["active_off"],
                 kw["max_file_size"], kw["now"], kw.get("io_type", 0))
    assert res.status == py["status"] and res.bad_file == py["bad_file"]
    if py["status"] != 0:
        return
    assert stream.tobytes() == py["stream"]
    assert [(int(p["fid"]), int(p["offset"]), int(p["entry_size"]), int(p["src_offset"]), int(p["src_file"]))
            for p in pos] == py["pos"]
    assert [(int(s["fid"]), int(s["file_off"]), int(s["stream_off"]), int(s["n_bytes"])) for s in segs] == \
        py["segments"]
    assert live.tolist() == py["live"]
    assert (res.end_fid, res.end_off) == (py["end_fid"], py["end_off"])
    assert res.n_live == sum(py["live"]) == int(stats["live_count"].sum())


def test_reference_writelogentry_positions():
    # db_test.go:197-229: entrySize 74 at (fid 1, off 0), (1, 74), then rollover to (2, 0)
    files, kw = MC.case_ref_writelogentry()
    res, stream, pos, segs, live, stats = run_c(files, kw)
    assert [(int(p["fid"]), int(p["offset"]), int(p["entry_size"])) for p in pos] == [(1, 0, 74), (1, 74, 74),
                                                                                        (2, 0, 74)]
    assert (res.end_fid, res.end_off) == (2, 74)


def test_reference_merge_shape():
    # db_test.go:64-109 shape: only key1's last Set lives in an archived file; key2's is in the active file
    files, kw = MC.case_ref_merge_shape()
    res, stream, pos, segs, live, stats = run_c(files, kw)
    assert res.n_records == 200 and res.n_live == 2 and res.n_emit == 1
    assert (int(pos[0]["fid"]), int(pos[0]["offset"])) == (kw["active_fid"], kw["active_off"])
    assert int(pos[0]["src_file"]) == 99 // 6 and int(pos[0]["src_offset"]) == (99 % 6) * 74


def test_generator_half_stale():
    imgs, n, ends = coracle.gen_merge(4, 1 << 20, 8000, 3, ksize=64, vsize=256)
    files = [(im, i, i < 3) for i, im in enumerate(imgs)]
    res, stream, pos, segs, live, stats = coracle.merge(files, 3, ends[3], 1 << 20, MC.NOW)
    assert res.n_records == n == 8000 and res.n_live == 4000
    assert all(int(s) == 332 for s in pos["entry_size"])


def test_golden_mix_reencodes_noncanonical():
    files, kw = MC.case_golden_mix()
    res, stream, pos, segs, live, stats = run_c(files, kw)
    src = {int(p["src_file"]) for p in pos}
    assert 1 in src and 2 in src  # noncanonical / noncanonical5 records were rewritten
    # every emitted record is canonical: decoding it gives hdr_size == enc_hdr_size and a valid CRC
    r, tup = coracle.scan(np.frombuffer(stream.tobytes() + bytes(64), np.uint8), 0, 0, 1)
    assert r.n_entries == res.n_emit
    assert np.array_equal(tup["hdr_size"], tup["enc_hdr_size"])
