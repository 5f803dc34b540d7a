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


@pytest.fixture(scope="module")
def gpu_engine():
    """A fresh engine (ldb_ctx) per GPU test module, destroyed at module end: the suite creates and
    destroys contexts in module order, the way a host process that opens and closes databases does
    (the fault this used to meet and its fix)."""
    import torch
    from lazydb_amd import Engine
    e = Engine(0)
    yield e
    torch.cuda.synchronize()
    e.close()
