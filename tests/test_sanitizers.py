"""ASan + UBSan over the CPU wave emulator (the engine's own phase code: ldb_engine.h, ldb_chain.h,
ldb_wave.h, ldb_pipeline.h, as tests/emu compiles them) and the C oracle: tests/san/san_main.cpp runs
both over every golden fixture (and ragged cuts of each), generated fixed / Zipf / reference-bench /
writer-mix logs and a corrupt one, under both IO rules, with the run prefix on and off, and compares
every tuple with the oracle. A sanitizer report aborts the run (halt_on_error)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_emulator_and_oracle_under_asan_ubsan():
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "san"), "run"], capture_output=True, text=True,
                       timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "0 mismatches" in out, out[-2000:]
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/clang++"), reason="no clang")
def test_sweep_tier_emulation_under_asan_ubsan():
    """The sweep tier's kernel code (ldb_sweep_kern.h) under the SIMT emulation (tests/emu/simt.h), built
    with clang and the same sanitizers, over the golden fixtures (one ragged cut each) and the generated
    logs, both IO rules, against the oracle (san_sweep: tests/san/Makefile)."""
    p = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "san"), "run_sweep"], capture_output=True,
                       text=True, timeout=900)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    assert "0 mismatches" in out, out[-2000:]
    assert "runtime error" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]
