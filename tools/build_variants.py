"""Build tuning variants of liblazydb_gpu.so (waves per workgroup, LDS ring depth, stamps, -D switches,
the library as of a git revision, backend scheduler options).

Usage: python tools/build_variants.py w8n2 w12n1 stamps git_<rev> def_NAME=V ...  -> lazydb_amd/_lib/var_<name>.so
Select one at run time with LAZYDB_GPU_LIB=<path>.
"""
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "lazydb_amd", "csrc", "ldb_scan.hip")
OUT = os.path.join(ROOT, "lazydb_amd", "_lib")


def build(name: str) -> str:
    defs = []
    m = re.fullmatch(r"w(\d+)n(\d+)", name)
    if m:
        defs = [f"-DLDB_WPB={m.group(1)}", f"-DLDB_NB={m.group(2)}"]
    elif name.startswith("git_"):   # the library as of a commit (A/B timing on one box)
        import tempfile
        rev = name[4:]
        tmp = tempfile.mkdtemp()
        for d in ("lazydb_amd/csrc", "include"):
            os.makedirs(os.path.join(tmp, d), exist_ok=True)
            for f in subprocess.run(["git", "-C", ROOT, "ls-tree", "--name-only", f"{rev}:{d}"], check=True,
                                    capture_output=True, text=True).stdout.split():
                with open(os.path.join(tmp, d, f), "wb") as fh:
                    fh.write(subprocess.run(["git", "-C", ROOT, "show", f"{rev}:{d}/{f}"], check=True,
                                            capture_output=True).stdout)
        out = os.path.join(OUT, f"var_{name}.so")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-Wno-unused-function", "-o", out, os.path.join(tmp, "lazydb_amd/csrc/ldb_scan.hip"),
                        *([m] if os.path.exists(m := os.path.join(tmp, "lazydb_amd/csrc/ldb_merge.hip")) else [])],
                       check=True)
        return out
    elif name.startswith("llvm_"):   # backend scheduling options (A/B of codegen only)
        opts = {"maxilp": ["-amdgpu-sched-strategy=max-ilp"], "iterilp": ["-amdgpu-sched-strategy=iterative-ilp"],
                "memclause": ["-amdgpu-sched-strategy=max-memory-clause"], "wavepri": ["-amdgpu-set-wave-priority"],
                "trackers": ["-amdgpu-use-amdgpu-trackers=1"], "relaxocc": ["-amdgpu-schedule-relaxed-occupancy"],
                "bias100": ["-amdgpu-schedule-metric-bias=100"], "bias0": ["-amdgpu-schedule-metric-bias=0"]}[name[5:]]
        defs = [x for o in opts for x in ("-mllvm", o)]
    elif name.startswith("def_"):   # def_NAME=VALUE[,NAME=VALUE...]: plain -D switches
        defs = ["-D" + d for d in name[4:].split(",")]
        name = re.sub(r"[^A-Za-z0-9_]", "_", name)
    elif name == "stamps":
        defs = ["-DLDB_STAMPS=1"]
    elif name == "stamps1":   # one wave per SIMD: phase stamps measure each wave's own critical path
        defs = ["-DLDB_STAMPS=1", "-DLDB_WPB=4", "-DLDB_NB=3", "-DLDB_BLOCKS_PER_CU=1"]   # 112 KB LDS: 1 block/CU
    else:
        raise SystemExit(f"unknown variant {name}")
    out = os.path.join(OUT, f"var_{name}.so")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                    "-Wno-unused-function", *defs, "-o", out, SRC, SRC.replace("ldb_scan.hip", "ldb_merge.hip")], check=True)
    return out


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    with ThreadPoolExecutor(4) as ex:
        for p in ex.map(build, sys.argv[1:]):
            print(p)
