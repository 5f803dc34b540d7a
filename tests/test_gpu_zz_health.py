"""Runs last in `pytest -m gpu`: the process is still healthy after every other GPU module.

Regression guard for DESIGN.md §7a: small host-to-device copies and a scan right after the parity
module's multi-GiB images and downloads."""
import numpy as np
import pytest

from oracle import coracle

pytestmark = pytest.mark.gpu


def test_copies_and_scan_after_the_suite():
    import torch
    from lazydb_amd import Engine
    torch.cuda.synchronize()
    for n in (1 << 10, 1 << 16, 3 << 20):
        a = np.arange(n, dtype=np.uint64).astype(np.uint8)
        d = torch.from_numpy(a).to("cuda:0")
        assert np.array_equal(d.cpu().numpy(), a)
    img, n, end = coracle.gen_log(1 << 20, 9, ksize=32, vsize=100)
    eng = Engine(0)
    res, tup = eng.scan_dev(torch.from_numpy(img).to("cuda:0"))
    ref, rt = coracle.scan(img)
    assert (res.status, res.end_off, res.n_entries) == (ref.status, ref.end_off, ref.n_entries)
    assert np.array_equal(tup["pos"], rt["pos"])
    eng.close()
