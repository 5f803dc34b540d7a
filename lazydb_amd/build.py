"""In-tree build of liblazydb_gpu.so (hipcc, gfx950) — no JIT cache, so the .so travels with the repo."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SRCS = [os.path.join(HERE, "csrc", f) for f in ("ldb_scan.hip", "ldb_merge.hip")]
OUT = os.path.join(HERE, "_lib", "liblazydb_gpu.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False) -> str:
    csrc = os.path.join(HERE, "csrc")
    deps = [os.path.join(csrc, f) for f in os.listdir(csrc)] + [os.path.join(ROOT, "include", "lazydb_gpu.h")]
    if force or _stale(OUT, deps):
        os.makedirs(os.path.dirname(OUT), exist_ok=True)
        # the translation units in parallel (each carries its own code object), then one link
        flags = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function"]
        objs = [os.path.join(os.path.dirname(OUT), os.path.basename(s) + ".o") for s in SRCS]
        procs = [subprocess.Popen([*flags, "-c", "-o", o, s]) for s, o in zip(SRCS, objs)]
        rcs = [pr.wait() for pr in procs]
        if any(rcs):
            raise subprocess.CalledProcessError(max(rcs, key=abs), "hipcc")
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-o", OUT, *objs], check=True)
        for o in objs:
            os.remove(o)
    return OUT


def build_all(force: bool = False) -> None:
    build_lib(force)
