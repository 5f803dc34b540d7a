import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblazydb_gpu.so on cuda:0)")
    config.addinivalue_line("markers", "slow: multi-GiB parity cases")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        meta = json.load(f)
    imgs = {}
    for m in meta:
        if m["name"] not in imgs:
            with open(os.path.join(ROOT, "tests", "golden", m["name"] + ".bin"), "rb") as f:
                imgs[m["name"]] = f.read()
    return meta, imgs


@pytest.fixture(scope="session")
def gpu_engine():
    """One engine (ldb_ctx) for every GPU test module of the session: the modules used to create and
    destroy one each, and a fresh context after a destroyed one met a GPU memory fault in its first
    test."""
    import torch
    from lazydb_amd import Engine
    e = Engine(0)
    yield e
    torch.cuda.synchronize()
    e.close()
