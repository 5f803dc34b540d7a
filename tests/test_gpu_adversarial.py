"""GPU parity on adversarial logs (DESIGN.md §5 "Adversarial logs", §3.3 two-phase k_repair).

Blocks of whole entries from the golden-fixture generators (tools/adversarial.py) are tiled to a
few MiB, so most region links break (values holding valid entries, headers with every field varied)
or the lean path sees Tx.Commit's 10-byte TxID varints, and the scan must still equal the C oracle
bit for bit: status, end_off, count and every index tuple, under both IOController rules. A corrupt
byte in the middle of the tiled image checks the repair's chain against a CRC stop as well.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from oracle import coracle  # noqa: E402  checker only

pytestmark = pytest.mark.gpu

CASES = ["embedded", "mixed", "binary", "txlog", "tiny", "big"]


@pytest.fixture(scope="module")
def eng():
    from lazydb_amd import Engine
    e = Engine(0)
    yield e
    e.close()


def _tiled(case: str, mib: int) -> np.ndarray:
    import adversarial as A
    b = A.block(case)
    n = max(1, (mib << 20) // b.size)
    return np.concatenate([np.tile(b, n), np.zeros(64, np.uint8)])


def _check(eng, img: np.ndarray, io: int):
    import torch
    d = torch.from_numpy(img).to("cuda:0")
    res, tup = eng.scan_dev(d, io_type=io, cap=img.size // 10 + 16)
    ref, rt = coracle.scan(img, io)
    assert (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries)
    assert np.array_equal(tup["pos"], rt["pos"])
    assert np.array_equal(tup["k_size"], rt["k_size"]) and np.array_equal(tup["v_size"], rt["v_size"])
    return res


@pytest.mark.parametrize("case", CASES)
def test_adversarial_parity(eng, case):
    img = _tiled(case, 24)
    for io in (0, 1):
        _check(eng, img, io)


@pytest.mark.parametrize("case", ["embedded", "mixed", "txlog"])
def test_adversarial_corrupt_middle(eng, case):
    img = _tiled(case, 12)
    img[img.size // 2] ^= 0x5A   # a CRC (or decode) stop in the middle of a repaired chain
    res = _check(eng, img, 0)
    assert res.end_off <= img.size // 2 + 1


def test_txlog_lean_path(eng):
    """Tx.Commit's snowflake TxIDs (9-10 byte varints) stay on the lean path: no repairs."""
    res = _check(eng, _tiled("txlog", 24), 0)
    assert res.n_repairs == 0 and res.n_broken == 0
    assert res.n_fast >= res.n_regions * 8 // 10
