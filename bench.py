"""Benchmark: device-resident LazyDB log decode + CRC32 on MI355X.

One "step" = one full replay scan (ReadLogEntry chain of index.go:84-95: decode,
CRC-32 verify, index tuples) of one log-file image already resident in HBM, per GPU.

Default workload, at every N = BASELINE config 4's per-GPU file: one 4 GiB log file of
64-B key / 256-B value entries per GPU (seed 10 + rank, FileIO bound) -> 12 936 648
entries, 4 294 967 136 valid bytes each. The same per-GPU file at N = 1, 2, 4, 8 makes
the 1 -> N curve comparable (weak scaling: independent files, index.go:68-95).
At N = 1 the line also carries `legs`: BASELINE config 2 (1 GiB) and config 3
(8 GiB, Zipf values), each timed the same way (GiB/s, kernel ms, roofline frac).

Multi-GPU: `python bench.py --gpus N` spawns N rank processes itself (before anything
touches the GPU); `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`
works as well. No collective on the scan path; after the timed scans the index tuples
are gathered to rank 0 with one RCCL gather, reported separately as `gather`.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=4, choices=[1, 2, 3, 4, 5],
                    help="BASELINE config: 1 = 500K entries 64/256 in a 512 MiB preallocated file (reopen); 2 = 1 GiB fixed 64/256; 3 = 8 GiB Zipf values; 4 = 4 GiB per GPU; "
                         "5 = merge/GC of 16 x 256 MiB files, half the records stale (a separate bench line)")
    ap.add_argument("--io", type=int, default=0, help="0 FileIO bound rule, 1 Mmap")
    ap.add_argument("--kind", type=int, default=0, help="0 index tuples (16 B), 1 full entries (48 B)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--gather", type=int, default=1)
    ap.add_argument("--cpu-sample-mib", type=int, default=1024)
    ap.add_argument("--xmerge", action="store_true",
                    help="config 5 as ONE 16-file set split over the ranks in fid blocks (cross-GPU merge)")
    ap.add_argument("--xhash", action="store_true",
                    help="with --xmerge/--xsim: the hash-partitioned liveness (route, owner resolve, apply)")
    ap.add_argument("--xsim", type=int, default=0,
                    help="config 5 --xmerge: play K ranks in this one process and time each rank's phases")
    ap.add_argument("--e2e", type=int, default=3, help="iterations of the PCIe-inclusive host-API leg (0: skip)")
    ap.add_argument("--legs", default="1,2,3,w,5",
                    help="extra single-GPU configs timed after the main line at N = 1 (comma list; '' = none): "
                         "1 the reference bench's log (Mmap), 2, 3, w the writer-realistic mix, 5 the merge")
    ap.add_argument("--leg-steps", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="after the W warm-up steps, keep stepping (untimed) until this much wall time has passed: "
                         "the GPU's clocks move for the first ~20 ms of sustained load (a kernel trace of 64 "
                         "back-to-back config-4 scans: k_uniform 0.74 -> 0.95 -> 0.755 ms, profiles/r04_dvfs_transient.txt), "
                         "so K timed steps right after 5 warm-up steps measure the transient, not the rate")
    ap.add_argument("--pmc", type=int, default=1,
                    help="measure roofline.traffic in this run: a rocprofv3 --pmc FETCH_SIZE child process scans "
                         "the same image (N = 1, rank 0; 0: skip)")
    ap.add_argument("--pmc-child", default="", help=argparse.SUPPRESS)
    ap.add_argument("--rehearse-launch", action="store_true",
                    help="launcher self-test without a GPU: ranks rendezvous over gloo and report")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """`bench.py --gpus N` without a launcher: start N rank processes of this script (children, not
    an exec: this process never touches the GPU), one per GPU, with the torch.distributed env a
    torchrun launch would give them. Rank 0 prints the JSON line. Returns the exit code."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(args.gpus),
                   RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(args.gpus))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    for p in procs:
        c = p.wait()
        if c != 0 and rc == 0:
            rc = c
            for q in procs:   # one rank failed: the others would wait forever in a collective
                if q.poll() is None:
                    q.kill()
    return rc


def rehearse_launch(args):
    """Launcher self-test (tests/test_bench_launch.py): every rank joins a gloo group and rank 0
    prints the bench's JSON keys that depend on the launch."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([rank], dtype=torch.int64)
    seen = [torch.zeros_like(t) for _ in range(world)]
    if world > 1:
        dist.all_gather(seen, t)
    else:
        seen = [t]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_seen": [int(x.item()) for x in seen],
                          "local_ranks_distinct": True, "config": {"workload": "launcher rehearsal (no GPU)"}}))
    if world > 1:
        dist.destroy_process_group()


def make_image(cfg, rank: int):
    """Synthetic image of a bench config. Returns (img, entries, end_off, workload text, IO rule or None
    for the command line's)."""
    from oracle import coracle  # format producer (writeLogEntry restatement) for synthetic inputs
    io = None
    if cfg == 1:
        # BASELINE config 1 in the reference benchmark's own shape (bench/db_bench_test.go:17-36, :63-68):
        # 500 000 Sets of "bench_test_key_<i>" (16..21-B keys: the entry size changes at i = 10, 100, ...)
        # with 512-B alphabet values, in one file preallocated to MaxLogFileSize = 512 MiB, reopened under
        # the Mmap IOController (opts.IOType = 1: o + n >= len is EOF, iocontroller/mmap.go:46-52)
        img, n, end = coracle.gen_bench_log(512 << 20, 1 + rank, n_entries=500_000)
        wl = "reference bench log: 500K Sets, bench_test_key_<i> keys, 512B values, 512 MiB preallocated, Mmap rule"
        io = 1
    elif cfg == 2:
        img, n, end = coracle.gen_log(1 << 30, 1 + rank, ksize=64, vsize=256)
        wl = "1GiB log file, 64B key / 256B value (332B entries), FileIO bound"
    elif cfg == 3:
        img, n, end = coracle.gen_log(8 << 30, 2 + rank, ksize=64, value_mode=1, zipf_s=1.1, zipf_max=4096)
        wl = "8GiB log file, 64B key, value 16*Zipf(1.1,[1,4096]) B"
    elif cfg == "w":
        # what LazyDB's writers append, interleaved (str.go Set / SetEX / Delete, tx.go Commit): variable
        # keys and values, 10 % SetEX (5-byte ExpiredAt), 10 % SDelete, 10 % TxCommited
        img, n, end = coracle.gen_writer_log(1 << 30, 30 + rank)
        wl = "1GiB writer-realistic log: Set/SetEX/Delete/Tx.Commit mix, user:<id> keys, 8B-4KiB log-uniform values"
    else:
        img, n, end = coracle.gen_log(4 << 30, 10 + rank, ksize=64, vsize=256)
        wl = "4GiB log file per GPU, 64B key / 256B value"
    return img, n, end, wl, io


def _host_threads() -> int:
    """Host threads this process may use: its CPU affinity, capped by the box's share when the
    environment states one (OMP_NUM_THREADS is set to the per-GPU CPU share on the GPU boxes)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        n = min(n, int(cap))
    return max(n, 1)


def cpu_baseline(img, end, sample_mib: int):
    """CPU baselines on a bounded sample (the first `sample_mib` MiB of the same log, cut at an entry
    boundary), BASELINE.md's two restatements of the reference replay:
    * faithful port (the `value`): pread per header and per k+v, heap buffers, CRC verify, a second
      CRC for the EncodeEntry size (log_file.go:116-145, index.go:15-26), one thread, as index.go
      replays one file at a time per value type;
    * optimized port: the in-memory scan with carry-less-multiply CRC folding (Go amd64
      hash/crc32's algorithm class), on one thread and on every host thread this process may use,
      one file per thread (each thread scans its own pass over the sample)."""
    import ctypes as C
    import threading
    from oracle import coracle
    n_bytes = min(end, sample_mib << 20)
    # cut the sample at an entry boundary: scan the prefix with the in-memory port
    res, tup = coracle.scan(img[: n_bytes + 64], cap=0)
    cut = int(res.end_off) if res.end_off <= n_bytes else n_bytes
    with tempfile.NamedTemporaryFile(dir="/dev/shm" if os.path.isdir("/dev/shm") else None, delete=True) as f:
        f.write(img[:cut].tobytes())
        f.flush()
        fd = os.open(f.name, os.O_RDONLY)
        try:
            t0 = time.perf_counter()
            r, _ = coracle.scan_faithful(fd, cut, 0, 1, cap=0)
            dt = time.perf_counter() - t0
        finally:
            os.close(fd)
    sample = img[:cut]
    L = coracle.lib()

    def one_pass(out):
        rr = coracle.ScanResult()
        L.ldbo_scan(sample.ctypes.data, cut, 0, 1, 0, None, 0, C.byref(rr))   # ctypes drops the GIL
        out.append(rr)

    t0 = time.perf_counter()
    got = []
    one_pass(got)
    dt1 = time.perf_counter() - t0
    nt = _host_threads()
    got = []
    ths = [threading.Thread(target=one_pass, args=(got,)) for _ in range(nt)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dtn = time.perf_counter() - t0
    assert len(got) == nt and all(int(g.end_off) == cut for g in got)
    # every host thread ("1, and all host cores"): one pass per thread; the process's CPU
    # affinity / quota may give it fewer cores than the machine has, so both counts are recorded
    na = os.cpu_count() or 1
    got = []
    ths = [threading.Thread(target=one_pass, args=(got,)) for _ in range(na)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dta = time.perf_counter() - t0
    assert len(got) == na and all(int(g.end_off) == cut for g in got)
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = na
    return {"value": round(r.end_off / dt / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {cut} B ({r.n_entries} entries) of the same log, faithful pread/alloc/2xCRC replay port, "
                      f"1 thread",
            "mentries_per_s": round(r.n_entries / dt / 1e6, 3),
            "optimized_port": {"GiB_per_s": round(cut / dt1 / 2**30, 3), "cores": 1,
                               "mentries_per_s": round(r.n_entries / dt1 / 1e6, 3)},
            "optimized_port_host_share": {"GiB_per_s": round(nt * cut / dtn / 2**30, 3), "cores": nt,
                                          "of_host_threads": os.cpu_count(),
                                          "label": f"per-GPU host share ({nt} of {os.cpu_count()} threads: the box's "
                                                   f"CPU share for one GPU, OMP_NUM_THREADS), not all host cores",
                                          "mentries_per_s": round(nt * r.n_entries / dtn / 1e6, 3),
                                          "sample": f"{nt} threads, one {cut}-B file pass each"},
            "optimized_port_all_cores": {"GiB_per_s": round(na * cut / dta / 2**30, 3), "cores": na,
                                         "usable_cpus": usable,
                                         "label": f"all host threads ({na} threads, {usable} CPUs in this process's "
                                                  f"affinity; a CPU quota may cap them further)",
                                         "mentries_per_s": round(na * r.n_entries / dta / 1e6, 3),
                                         "sample": f"{na} threads, one {cut}-B file pass each"},
            "host_cpu": _cpu_model(), "host_nproc": os.cpu_count()}


def pmc_child(args):
    """Child of measure_traffic(), run under rocprofv3 --pmc: scan an image file a few times."""
    import numpy as np
    import torch
    from lazydb_amd import Engine
    path, cap = args.pmc_child.rsplit(":", 1)
    img = np.fromfile(path, dtype=np.uint8)
    eng = Engine(0)
    S = Resident(eng, img, int(cap), args.kind, torch.device("cuda:0"))
    eng.reserve(img.size)
    for _ in range(3):
        eng.scan_dev_async(S.d, fid=1, io_type=args.io, kind=args.kind, out=S.out, cap=S.cap, result=S.res)
    torch.cuda.synchronize()
    eng.close()


def measure_traffic(img, cap, args, kernel):
    """HBM bytes per launch of `kernel` (the dominant one), measured in this run: a child process scans the same image
    under `rocprofv3 --pmc FETCH_SIZE` (a counter-only pass, no other trace), and FETCH_SIZE is
    doubled, the gfx950 correction for wide streaming reads (MI355X_MICROARCH.md "HBM"). Counters
    cannot be read inside this process. Returns (bytes or None, how it was obtained)."""
    import csv
    import glob
    import shutil
    import subprocess
    if not args.pmc or not shutil.which("rocprofv3"):
        return None, "not measured (rocprofv3 absent or --pmc 0)"
    tmp = tempfile.mkdtemp(prefix="ldb_pmc_", dir="/tmp")
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else tmp
    path = os.path.join(shm, f"ldb_pmc_{os.getpid()}.bin")
    try:
        img.tofile(path)
        # the device path's instance only (k_uniform<false, false>, k_sweep<false>, k_region<false>): not k_uniform_fill
        tag = kernel + "<false"
        cmd = ["timeout", "-s", "KILL", "180", "rocprofv3", "--pmc", "FETCH_SIZE", "--kernel-include-regex",
               kernel + "<false", "-d", tmp, "-o", "pmc", "-f", "csv", "--", sys.executable, os.path.abspath(__file__),
               "--pmc-child", f"{path}:{cap}", "--io", str(args.io), "--kind", str(args.kind)]
        p = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
        per = {}
        for f in glob.glob(os.path.join(tmp, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if tag in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE":
                        key = r.get("Dispatch_Id") or r.get("Dispatch_ID") or r.get("Correlation_Id")
                        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
        if not per:
            return None, f"rocprofv3 child produced no {kernel} FETCH_SIZE (rc {p.returncode})"
        kib = sum(per.values()) / len(per)
        return int(kib * 1024 * 2), (f"measured in this run: rocprofv3 --pmc FETCH_SIZE over {len(per)} {kernel} "
                                     f"launches of the same image, x2 (gfx950 wide-read correction)")
    except Exception as e:   # the traffic figure is diagnostic: never fail the bench line over it
        return None, f"not measured ({type(e).__name__}: {e})"
    finally:
        if os.path.exists(path):
            os.unlink(path)
        shutil.rmtree(tmp, ignore_errors=True)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def init_dist(world: int, local: int) -> int:
    """One process per GPU over RCCL (backend "nccl"). LDB_BENCH_BACKEND=gloo rehearses the N>1
    path with ranks sharing the GPUs of a smaller box (device = local rank mod device count);
    the collectives then run on host copies (lazydb_amd.multi)."""
    import torch
    import torch.distributed as dist
    backend = os.environ.get("LDB_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    return local


def merge_leg(eng, args, dev):
    """BASELINE config 5 as a leg of the N = 1 line: the same merge as main_merge, verified against the
    oracle's merge (whose run is also the CPU baseline: the C port of Merge, one thread), then timed."""
    import numpy as np
    import torch
    from oracle import coracle   # format producer for the synthetic input; checker; CPU baseline
    now = 1_700_000_000
    imgs, n, ends = coracle.gen_merge(16, 256 << 20, 16 * 808_540, 3, ksize=64, vsize=256)
    files = [(torch.from_numpy(imgs[i]).to(dev), i + 1, i < 15) for i in range(16)]
    kw = dict(active_fid=16, active_off=ends[15], max_file_size=256 << 20, now=now)
    out = eng.merge_dev(files, **kw)
    r = out["result"]
    verified, cpu = None, None
    if not args.no_verify:
        t0 = time.perf_counter()
        ref, stream, pos, segs, live, stats = coracle.merge([(imgs[i], i + 1, i < 15) for i in range(16)], 16,
                                                            ends[15], 256 << 20, now)
        dt = time.perf_counter() - t0
        verified = bool((r.status, r.n_emit, r.emit_bytes, r.end_fid, r.end_off) ==
                        (ref.status, ref.n_emit, ref.emit_bytes, ref.end_fid, ref.end_off)
                        and out["pos"].tobytes() == pos.tobytes()
                        and torch.equal(out["stream"], torch.from_numpy(stream).to(dev)))
        cpu = {"value": round(sum(ends) / dt / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
               "sample": "the full 16-file set: oracle replay + map-based index + EncodeEntry rewrite, 1 thread "
                         "(the verification run, timed)"}
        del stream, pos, live
    caps = dict(stream_cap=int(r.emit_bytes) + 16, pos_cap=int(r.n_emit) + 16, seg_cap=64,
                live_cap=int(r.n_records) + 16, fetch_pos=False)
    for _ in range(2):
        eng.merge_dev(files, **kw, **caps)
    settle(lambda: eng.merge_dev(files, **kw, **caps), args.settle_ms)
    torch.cuda.synchronize()
    ph = np.zeros(3)
    steps = args.leg_steps
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.merge_dev(files, **kw, **caps)
        ph += np.array(eng.merge_timing())
    torch.cuda.synchronize()
    step = (time.perf_counter() - t0) / steps
    ph /= steps
    dev_ms = float(ph.sum())
    alg = sum(ends) + 2 * int(r.emit_bytes)   # replay read + compacted stream read and written
    leg = {"config": 5, "workload": "merge/GC: 16 log files x 256 MiB, 64B key / 256B value, 50% stale, 15 targets",
           "input_bytes": int(sum(ends)), "records": int(r.n_records), "emitted": int(r.n_emit),
           "emit_bytes": int(r.emit_bytes), "segments": int(r.n_segments), "steps": steps,
           "ms_per_step": round(step * 1e3, 4), "GiB_per_s": round(sum(ends) / step / 2**30, 3),
           "phases_ms": {"replay_scans": round(ph[0], 3), "liveness": round(ph[1], 3), "compaction": round(ph[2], 3)},
           "roofline": {"bound": "hbm", "kernel": "whole merge pipeline (device time)",
                        "achieved": round(alg / (dev_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                        "frac": round(alg / (dev_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4), "traffic": None,
                        "algorithmic_bytes_per_launch": alg,
                        "note": "algorithmic bytes = sum of end_off (replay read) + 2 x emitted bytes"},
           "verified_vs_oracle": verified, "cpu_baseline": cpu}
    del files, imgs
    torch.cuda.empty_cache()
    return leg


def main_merge(args):
    """BASELINE config 5: Merge/GC of one value type -- 16 log files x 256 MiB (64-B keys, 256-B values,
    every key written twice so exactly half the records are stale), 15 archived targets merged into
    the active file 16: replay scans + last-writer-wins liveness + compacted stream with rollover
    (db.go:383-427, 243-265, 473-523). One step = one ldb_merge_files_dev call over device-resident
    images. With N ranks each rank merges its own independent 16-file set (weak scaling); --xmerge
    splits ONE set over the ranks instead (main_xmerge)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = init_dist(world, local)
    dev = torch.device(f"cuda:{local}")
    from lazydb_amd import Engine
    from lazydb_amd import multi
    from oracle import coracle   # format producer for the synthetic input; checker
    now = 1_700_000_000
    imgs, n, ends = coracle.gen_merge(16, 256 << 20, 16 * 808_540, 3 + rank, ksize=64, vsize=256)
    files = [(torch.from_numpy(imgs[i]).to(dev), i + 1, i < 15) for i in range(16)]
    eng = Engine(local)
    kw = dict(active_fid=16, active_off=ends[15], max_file_size=256 << 20, now=now)
    out = eng.merge_dev(files, **kw)
    r = out["result"]
    verified = None
    if not args.no_verify:
        ref, stream, pos, segs, live, stats = coracle.merge([(imgs[i], i + 1, i < 15) for i in range(16)], 16,
                                                            ends[15], 256 << 20, now)
        verified = bool((r.status, r.n_emit, r.emit_bytes, r.end_fid, r.end_off) ==
                        (ref.status, ref.n_emit, ref.emit_bytes, ref.end_fid, ref.end_off)
                        and out["pos"].tobytes() == pos.tobytes()
                        and torch.equal(out["stream"], torch.from_numpy(stream).to(dev)))
        del stream, pos, live
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        t0 = time.perf_counter()
        coracle.merge([(imgs[i], i + 1, i < 15) for i in range(16)], 16, ends[15], 256 << 20, now)
        dt = time.perf_counter() - t0
        cpu = {"value": round(sum(ends) / dt / 2**30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
               "sample": "the full 16-file set: oracle replay + map-based index + EncodeEntry rewrite, 1 thread",
               "optimized_port_all_cores": {"GiB_per_s": round(na * cut / dta / 2**30, 3), "cores": na,
                                         "usable_cpus": usable,
                                         "label": f"all host threads ({na} threads, {usable} CPUs in this process's "
                                                  f"affinity; a CPU quota may cap them further)",
                                         "mentries_per_s": round(na * r.n_entries / dta / 1e6, 3),
                                         "sample": f"{na} threads, one {cut}-B file pass each"},
            "host_cpu": _cpu_model(), "host_nproc": os.cpu_count()}
    caps = dict(stream_cap=int(r.emit_bytes) + 16, pos_cap=int(r.n_emit) + 16, seg_cap=64,
                live_cap=int(r.n_records) + 16, fetch_pos=False)
    for _ in range(args.warmup):
        eng.merge_dev(files, **kw, **caps)
    settle(lambda: eng.merge_dev(files, **kw, **caps), args.settle_ms)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ph = np.zeros(3)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.merge_dev(files, **kw, **caps)
        ph += np.array(eng.merge_timing())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = multi.max_over_ranks(time.perf_counter() - t0, dev)
    ph /= args.steps
    in_bytes = sum(ends)
    tot_in = multi.sum_over_ranks([in_bytes], dev)[0]
    if rank == 0:
        step = t / args.steps
        dev_ms = float(ph.sum())
        alg = in_bytes + 2 * int(r.emit_bytes)   # replay read + compacted stream read and written
        print(json.dumps({
            "metric": "merge/GC decode+CRC32+liveness+compaction: input GiB/s (BASELINE config 5)",
            "value": round(tot_in / step / 2**30, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (writeLogEntry format, every key written twice)",
            "config": {"workload": "16 log files x 256 MiB, 64B key / 256B value, 50% stale, 15 targets",
                       "records": int(r.n_records), "live": int(r.n_live), "emitted": int(r.n_emit),
                       "emit_bytes": int(r.emit_bytes), "segments": int(r.n_segments),
                       "parallelism": f"one 16-file set per GPU x{world}"},
            "phases_ms": {"replay_scans": round(ph[0], 3), "liveness": round(ph[1], 3),
                          "compaction": round(ph[2], 3)},
            "roofline": {"bound": "hbm", "kernel": "whole merge pipeline (device time)",
                         "achieved": round(alg / (dev_ms * 1e-3) / 1e9, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                         "frac": round(alg / (dev_ms * 1e-3) / 1e9 / PEAK_HBM_GBS, 4), "traffic": None,
                         "algorithmic_bytes_per_launch": alg},
            "verified_vs_oracle": verified, "cpu_baseline": cpu}))
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def main_xmerge(args):
    """BASELINE config 5 over N GPUs as ONE merge: the 16-file set is split in contiguous fid blocks,
    one per rank (lazydb_amd/xmerge.py: summary all-gather, per-rank ldb_merge_files_dev, global
    rollover by ldb_merge_repack_dev). One step = one merge_distributed call; value = the set's
    input bytes / step time (strong scaling: the total work is fixed). --xsim K plays K ranks in this
    process, times each rank's phases on its own and reports the critical path (no exchange cost)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = init_dist(world, local)
    dev = torch.device(f"cuda:{local}")
    from lazydb_amd import Engine
    from lazydb_amd import multi
    from lazydb_amd import xmerge as X
    from oracle import coracle   # format producer for the synthetic input; checker
    now = 1_700_000_000
    imgs, n, ends = coracle.gen_merge(16, 256 << 20, 16 * 808_540, 3, ksize=64, vsize=256)
    kw = dict(active_fid=16, active_off=ends[15], max_file_size=256 << 20, now=now)
    eng = Engine(local)
    sim = args.xsim
    nr = sim if sim else world
    blocks = [list(b) for b in np.array_split(np.arange(16), nr)]
    mine = blocks[rank] if not sim else list(range(16))
    dfiles = {i: (torch.from_numpy(imgs[i]).to(dev), i + 1, i < 15) for i in mine}
    in_bytes = sum(ends)
    ref = None if args.no_verify else coracle.merge([(imgs[i], i + 1, i < 15) for i in range(16)], 16, ends[15],
                                                    256 << 20, now)

    def sync():
        torch.cuda.synchronize()

    if sim and args.xhash:
        engs = [eng] + [Engine(local) for _ in range(nr - 1)]
        names = ["route", "resolve", "apply", "place"]
        ph = np.zeros((nr, len(names)))
        cur = {"on": False}

        def timer(r, phase, fn):
            sync()
            t0 = time.perf_counter()
            out = fn()
            sync()
            if cur["on"]:
                ph[r, names.index(phase)] += time.perf_counter() - t0
            return out

        own = [[dfiles[i] for i in b] for b in blocks]
        for step in range(args.warmup + args.steps):
            cur["on"] = step >= args.warmup
            parts, places = X.hashed_sim(engs, own, kw["active_fid"], kw["active_off"], kw["max_file_size"],
                                         kw["now"], timer=timer, fetch_pos=False)
        ph /= args.steps
        verified = None
        if ref is not None:
            verified = bool(b"".join(p["stream"].cpu().numpy().tobytes() for p in parts) == ref[1].tobytes()
                            and places[-1]["end"] == (ref[0].end_fid, ref[0].end_off))
        crit = float(ph.max(axis=0).sum())
        # bytes that cross between ranks: route records + keys to other owners, one flag byte back each
        xbytes = 0
        for r in range(nr):
            ro = X.route_phase(engs[r], own[r], nr)
            for o in range(nr):
                if o != r:
                    xbytes += ro["rec_splits"][o] + ro["key_splits"][o] + int(ro["counts"][o])
        print(json.dumps({
            "metric": "merge/GC decode+CRC32+liveness+compaction: input GiB/s (BASELINE config 5), simulated ranks, "
                      "hash-partitioned liveness",
            "simulated_ranks": nr, "steps": args.steps, "warmup": args.warmup,
            "per_rank_ms": {k: [round(x * 1e3, 3) for x in ph[:, i]] for i, k in enumerate(names)},
            "critical_path_ms": round(crit * 1e3, 3),
            "est_GiB_per_s_without_exchange": round(in_bytes / crit / 2**30, 3),
            "exchange_bytes_between_ranks": xbytes,
            "exchange_ms_at_xgmi_7x153GBps_per_gpu": round(xbytes / nr / (7 * 153e9) * 1e3, 3),
            "verified_vs_oracle": verified}))
        for e in engs:
            e.close()
        return
    if sim:
        ph = np.zeros((nr, 3))
        verified = None
        for step in range(args.warmup + args.steps):
            own = [[dfiles[i] for i in b] for b in blocks]
            summ, parts, places = [], [], []
            for r in range(nr):
                sync(); t0 = time.perf_counter()
                summ.append(X.rank_summary(eng, own[r])[0] if r > 0 else None)   # rank 0's is never read
                sync(); ph[r, 0] += (time.perf_counter() - t0) if step >= args.warmup else 0
            for r in range(nr):
                sync(); t0 = time.perf_counter()
                parts.append(X.rank_merge(eng, own[r], summ[r + 1:], X.summary_fid_base(16) + r + 1, **kw))
                sync(); ph[r, 1] += (time.perf_counter() - t0) if step >= args.warmup else 0
            sizes = [X.entry_sizes(eng, p) for p in parts]
            for r in range(nr):
                sync(); t0 = time.perf_counter()
                places.append(X.rank_place(eng, parts[r], torch.cat(sizes[:r]) if r else None, kw["active_fid"],
                                           kw["active_off"], kw["max_file_size"], fetch_pos=False))
                sync(); ph[r, 2] += (time.perf_counter() - t0) if step >= args.warmup else 0
        ph /= args.steps
        if ref is not None:
            verified = bool(b"".join(p["stream"].cpu().numpy().tobytes() for p in parts) == ref[1].tobytes()
                            and places[-1]["end"] == (ref[0].end_fid, ref[0].end_off))
        crit = float(ph.max(axis=0).sum())
        xbytes = sum(int(s.numel()) for s in summ if s is not None)
        print(json.dumps({
            "metric": "merge/GC decode+CRC32+liveness+compaction: input GiB/s (BASELINE config 5), simulated ranks",
            "simulated_ranks": nr, "steps": args.steps, "warmup": args.warmup,
            "per_rank_ms": {"summary": [round(x * 1e3, 3) for x in ph[:, 0]],
                            "merge": [round(x * 1e3, 3) for x in ph[:, 1]],
                            "place": [round(x * 1e3, 3) for x in ph[:, 2]]},
            "critical_path_ms": round(crit * 1e3, 3),
            "est_GiB_per_s_without_exchange": round(in_bytes / crit / 2**30, 3),
            "summary_bytes_all_gathered": xbytes, "verified_vs_oracle": verified}))
        eng.close()
        return
    files = [dfiles[i] for i in mine]

    def step_once():
        if world > 1 and args.xhash:
            return X.merge_hashed_distributed(eng, files, **kw, fetch_pos=False)
        return (X.merge_distributed(eng, files, 16, **kw, fetch_pos=False) if world > 1
                else X.merge_distributed_single(eng, files, **kw, fetch_pos=False))

    out = step_once()
    verified = None
    if ref is not None:
        got = multi.gather_tuples(out["stream"]) if world > 1 else [out["stream"]]
        if rank == 0:
            verified = bool(b"".join(g.cpu().numpy().tobytes() for g in got) == ref[1].tobytes())
        if world > 1:
            ends_ok = torch.tensor([int(out["end"] == (ref[0].end_fid, ref[0].end_off)) if rank == world - 1 else 1],
                                   device=multi.coll_device(dev))
            dist.all_reduce(ends_ok, op=dist.ReduceOp.MIN)
            verified = bool(verified and int(ends_ok.item())) if rank == 0 else verified
    for _ in range(args.warmup):
        step_once()
    for _ in range(8 if args.settle_ms > 0 else 0):   # a fixed count: step_once holds collectives, so every
        step_once()                                    # rank must take the same number of steps
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_once()
    sync()
    if world > 1:
        dist.barrier()
    t = multi.max_over_ranks(time.perf_counter() - t0, dev)
    if rank == 0:
        step = t / args.steps
        print(json.dumps({
            "metric": "merge/GC decode+CRC32+liveness+compaction: input GiB/s (BASELINE config 5), one set over N GPUs",
            "value": round(in_bytes / step / 2**30, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(step * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (writeLogEntry format, every key written twice)",
            "config": {"workload": "16 log files x 256 MiB, 64B key / 256B value, 50% stale, 15 targets",
                       "parallelism": f"fid blocks over {world} GPU(s), " + (
                           "hash-partitioned liveness (2 all-to-alls)" if args.xhash else "summary all-gather") +
                       " + rollover chain"},
            "verified_vs_oracle": verified}))
    eng.close()
    if world > 1:
        dist.destroy_process_group()


def settle(step, ms: float, max_steps: int = 2000):
    """Untimed steps after the warm-up until `ms` of wall time has passed (at least one synchronised
    round): the device's clocks settle after the first ~20 ms of back-to-back launches (DVFS; see
    --settle-ms). Steps are enqueued in rounds of 8 and each round is synchronised, so the host never
    runs far ahead of the device."""
    import torch
    if ms <= 0:
        return 0
    t0, n = time.perf_counter(), 0
    while n < max_steps:
        for _ in range(8):
            step()
        n += 8
        torch.cuda.synchronize()
        if (time.perf_counter() - t0) * 1e3 >= ms:
            break
    settle.last_steps = n
    return n


settle.last_steps = 0


class Resident:
    """One log-file image in HBM with its output tuple array and result slot."""

    def __init__(self, eng, img, cap, kind, dev):
        import torch
        self.d = torch.from_numpy(img).to(dev)
        self.cap = cap
        self.out = eng.alloc_out(cap, kind)
        self.res = eng.alloc_result()


def timed_scans(eng, S, fid, args, steps, world, stream):
    """K device-resident scans of one image between barrier + synchronize: the headline wall time,
    with no instrumentation inside the pipelines. Then K more with HIP events recorded around the
    kernels on the scan stream, for the per-kernel split (an event record between two kernels adds a
    few microseconds of gap, so it stays out of the headline pass). Returns (wall seconds, avg
    k_uniform ms, avg k_region ms, avg pipeline ms); timed_scans.sweep_ms: avg k_sweep ms; timed_scans.phases:
    the phases after the run prefix (device clock)."""
    import torch
    import torch.distributed as dist

    def step():
        eng.scan_dev_async(S.d, fid=fid, io_type=S.io, kind=args.kind, out=S.out, cap=S.cap, result=S.res,
                           stream=stream)

    for _ in range(args.warmup):
        step()
    settle(step, args.settle_ms)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    timed_scans.enqueue_ms = (time.perf_counter() - t0) * 1e3   # host time to enqueue the K steps (diagnostic)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    # the median of >= 20 event-timed iterations (one event pair per scan on its stream;
    # reported beside the contract's wall-clock value)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(max(steps, 20))]
    for a, b in evs:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    med_ms = statistics.median(a.elapsed_time(b) for a, b in evs)
    eng.timing(1)
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ph = eng.timing_tail()   # (before timing_split, which resets the accumulators)
    timed_scans.sweep_ms = eng.timing_sweep()[0]
    run_ms, main_ms, total_ms, _ = eng.timing_split(0)
    timed_scans.phases = {k: round(v, 4) for k, v in zip(TAIL_PHASES, ph)}
    timed_scans.median_ms = med_ms
    timed_scans.median_iters = len(evs)
    return t, run_ms, main_ms, total_ms


TAIL_PHASES = ("sweep", "sweep_check", "regions", "links", "repair", "combine", "compact")


def dominant_kernel(S, r, kind, run_ms, main_ms, sweep_ms=0.0):
    """The scan's dominant kernel and its algorithmic bytes per launch (the bytes of
    the accepted entries it verified). k_uniform (the run prefix) verified entries [0, n_run), i.e.
    bytes [0, x0); k_sweep (the sweep tier, ldb_sweep.h) the next n_sweep, bytes [x0, x1); k_region
    (the region pipeline) the rest, [x1, end_off)."""
    n_run, n_sw, n, end = int(r.n_run), int(r.n_sweep), int(r.n_entries), int(r.end_off)
    tsz = 16 if kind == 0 else 48

    def start_of(k):   # image offset of entry k (end_off past the last one)
        if k >= n:
            return end
        return int.from_bytes(S.out[k * tsz: k * tsz + 8].cpu().numpy().tobytes(), "little") & ((1 << 40) - 1)
    x0 = start_of(n_run) if n_run else 0
    x1 = start_of(n_run + n_sw) if n_sw else x0
    best = max((run_ms, "k_uniform", x0), (sweep_ms, "k_sweep", x1 - x0), (main_ms, "k_region", end - x1))
    return best[1], best[2], best[0]


def prepare(eng, cfg, rank, args, dev, verify: bool):
    """Synthetic image of config `cfg` on the device plus its output buffers; one scan checked
    against the oracle before anything is timed. Returns (host image, device image, result, verified,
    workload text)."""
    import torch
    from lazydb_amd import _native as N
    img, n_expect, end_expect, workload, io = make_image(cfg, rank)
    S_io = args.io if io is None else io
    cap = n_expect + 1024
    S = Resident(eng, img, cap, args.kind, dev)
    S.io = S_io
    eng.reserve(img.size)
    stream = torch.cuda.current_stream(dev)
    eng.scan_dev_async(S.d, fid=1 + rank, io_type=S_io, kind=args.kind, out=S.out, cap=cap, result=S.res,
                       stream=stream)
    torch.cuda.synchronize()
    r = N.ScanResult.from_buffer_copy(S.res.cpu().numpy().tobytes())
    verified = None
    if verify:
        from oracle import coracle   # checker only
        ref, rt = coracle.scan(img, S_io, fid=1 + rank, tuple_kind=args.kind, cap=cap)
        n = int(min(r.n_entries, cap))
        got = S.out[: n * (16 if args.kind == 0 else 48)].cpu().numpy().tobytes()
        verified = (r.status, r.end_off, r.n_entries) == (ref.status, ref.end_off, ref.n_entries) and \
            got == rt.tobytes()
        del rt
    return img, S, r, verified, workload, end_expect


def run_leg(eng, cfg, args, dev):
    """One extra single-GPU config (N = 1 only): the same timed scans as the main line."""
    import torch
    img, S, r, verified, workload, _ = prepare(eng, cfg, 0, args, dev, not args.no_verify)
    t, run_ms, main_ms, total_ms = timed_scans(eng, S, 1, args, args.leg_steps, 1, torch.cuda.current_stream(dev))
    kname, kbytes, kms = dominant_kernel(S, r, args.kind, run_ms, main_ms, timed_scans.sweep_ms)
    step = t / args.leg_steps
    achieved = kbytes / (kms * 1e-3) / 1e9 if kms > 0 else None
    leg = {"config": cfg, "workload": workload, "file_bytes": int(img.size), "bytes_scanned": int(r.end_off),
           "entries": int(r.n_entries), "steps": args.leg_steps, "ms_per_step": round(step * 1e3, 4),
           "GiB_per_s": round(int(r.end_off) / step / 2**30, 3),
           "mentries_per_s": round(int(r.n_entries) / step / 1e6, 2),
           "median_event_ms": round(timed_scans.median_ms, 4),
           "GiB_per_s_median": round(int(r.end_off) / (timed_scans.median_ms * 1e-3) / 2**30, 3),
           "k_uniform_ms": round(run_ms, 4), "k_sweep_ms": round(timed_scans.sweep_ms, 4), "k_region_ms": round(main_ms, 4),
           "tail_phases_ms": timed_scans.phases,
           "pipeline_ms": round(total_ms, 4),
           "run_entries": int(r.n_run), "sweep_entries": int(r.n_sweep), "roofline_kernel": kname, "roofline_bytes": kbytes,
           "roofline_frac": round(achieved / PEAK_HBM_GBS, 4) if achieved else None,
           "status": int(r.status), "fast_regions": int(r.n_fast), "regions": int(r.n_regions),
           "regions_rerun": int(r.n_repairs), "io_type": "FileIO" if S.io == 0 else "Mmap",
           "verified_vs_oracle": verified}
    del S, img
    torch.cuda.empty_cache()
    return leg


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    if args.rehearse_launch:
        return rehearse_launch(args)
    if args.pmc_child:
        return pmc_child(args)
    if args.config == 5 and (args.xmerge or args.xsim):
        return main_xmerge(args)
    if args.config == 5:
        return main_merge(args)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = init_dist(world, local)
    dev = torch.device(f"cuda:{local}")

    from lazydb_amd import Engine
    from lazydb_amd import _native as N

    eng = Engine(local)
    img, S, r, verified, workload, end_expect = prepare(eng, args.config, rank, args, dev, not args.no_verify)
    stream = torch.cuda.current_stream(dev)
    t, run_ms, main_ms, total_ms = timed_scans(eng, S, 1 + rank, args, args.steps, world, stream)
    med_ms, med_iters = timed_scans.median_ms, timed_scans.median_iters
    kname, kbytes, kms = dominant_kernel(S, r, args.kind, run_ms, main_ms, timed_scans.sweep_ms)
    # practical HBM-read ceiling on this box: a read-only reduction over the same image, after the
    # timed region
    ceiling = eng.read_ceiling(S.d, 20) if rank == 0 else None

    bytes_scanned = int(r.end_off)
    entries = int(r.n_entries)
    from lazydb_amd import multi
    t_max = multi.max_over_ranks(t, dev)
    tot_bytes, tot_entries = multi.sum_over_ranks([bytes_scanned, entries], dev)
    all_ok = multi.sum_over_ranks([1 if verified else 0], dev)[0] if verified is not None else None
    gather = None
    if world > 1 and args.gather:
        # the north star's single exchange: every rank's index tuples to rank 0 over RCCL/xGMI
        mine = S.out[: entries * (16 if args.kind == 0 else 48)]
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        got = multi.gather_tuples(mine)
        torch.cuda.synchronize()
        gt = multi.max_over_ranks(time.perf_counter() - g0, dev)
        if rank == 0:
            tot = sum(int(x.numel()) for x in got)
            moved = multi.gather_tuples.last_bytes
            gather = {"bytes_to_rank0": tot, "bytes_moved": moved, "ms": round(gt * 1e3, 3),
                      "GB_per_s": round(moved / gt / 1e9, 2), "backend": dist.get_backend(),
                      "method": "gatherv: all_gather of the counts, then batched isend/irecv of exactly those bytes",
                      "exact": tot == int(tot_entries) * (16 if args.kind == 0 else 48)}
            del got
    e2e = None
    cap = S.cap
    if world == 1 and args.e2e > 0:
        # PCIe-inclusive rate of the host-pointer API (ldb_scan_file: H2D of the image from pageable
        # host memory, scan, D2H of the tuples) -- recorded for DESIGN.md, never the bench value
        res_h, _ = eng.scan_host(img, fid=1, io_type=args.io, kind=args.kind, cap=cap)
        t0e = time.perf_counter()
        for _ in range(args.e2e):
            res_h, _ = eng.scan_host(img, fid=1, io_type=args.io, kind=args.kind, cap=cap)
        te = (time.perf_counter() - t0e) / args.e2e
        e2e = {"GiB_per_s": round(int(res_h.end_off) / te / 2**30, 3), "ms": round(te * 1e3, 2),
               "path": "ldb_scan_file: pageable host image -> H2D -> scan -> D2H tuples",
               "status_matches": int(res_h.status) == int(r.status) and int(res_h.n_entries) == entries}
        # the same with the image and the tuple array page-locked once (ldb_host_register, as a caller
        # holding an mmap'd file and a reused tuple buffer would): the chunks go up by DMA at PCIe
        # rate, the run prefix verifies each as it lands, and the kernels write the tuples in place
        # 
        import numpy as np
        hout = np.zeros(cap, dtype=N.INDEX_TUPLE if args.kind == 0 else N.ENTRY_TUPLE)   # the caller's reused array
        eng.host_register(img)
        eng.host_register(hout)
        try:
            eng.scan_host(img, fid=1, io_type=args.io, kind=args.kind, out=hout)
            t0e = time.perf_counter()
            for _ in range(args.e2e):
                res_h, _ = eng.scan_host(img, fid=1, io_type=args.io, kind=args.kind, out=hout)
            te = (time.perf_counter() - t0e) / args.e2e
        finally:
            eng.host_unregister(hout)
            eng.host_unregister(img)
        e2e["registered"] = {"GiB_per_s": round(int(res_h.end_off) / te / 2**30, 3), "ms": round(te * 1e3, 2),
                             "GB_per_s": round(int(res_h.end_off) / te / 1e9, 2),
                             "path": "ldb_scan_file, page-locked image and tuple array: 64 MiB chunks over 2 "
                                     "DMA streams, run prefix verified per chunk as it lands, tuples written in place",
                             "status_matches": int(res_h.n_entries) == entries}
        e2e["GB_per_s"] = round(int(r.end_off) / (e2e["ms"] * 1e-3) / 1e9, 2)
    ms_step = t_max / args.steps * 1e3
    value = tot_bytes / (t_max / args.steps) / 2**30
    # every rank's dominant kernel, so the N > 1 line carries a roofline per rank (one all-gather)
    per_rank = multi.gather_floats([kbytes, kms, run_ms, main_ms, total_ms, t / args.steps * 1e3], dev)
    traffic, traffic_src = (measure_traffic(img, cap, args, kname) if rank == 0 and args.io == 0
                            else (None, "not measured (Mmap rule)"))
    cpu = None
    if rank == 0 and not args.no_cpu:
        # N > 1: a quarter of the sample (rank 0's host share; the other ranks wait at the final barrier)
        cpu = cpu_baseline(img, end_expect, args.cpu_sample_mib if world == 1 else max(64, args.cpu_sample_mib // 4))
    legs = []
    if world == 1 and args.legs:
        del S
        torch.cuda.empty_cache()
        for tok in [x.strip() for x in args.legs.split(",") if x.strip()]:
            cfg = tok if tok == "w" else int(tok)
            if cfg == 5:
                legs.append(merge_leg(eng, args, dev))
            elif cfg != args.config and cfg in (1, 2, 3, 4, "w"):
                legs.append(run_leg(eng, cfg, args, dev))
    if rank == 0:
        achieved = kbytes / (kms * 1e-3) / 1e9 if kms > 0 else None
        line = {
            "metric": "device-resident log decode+CRC32: GiB/s and Mentries/s at 1/2/4/8 MI355X",
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (LazyDB writeLogEntry format, splitmix64 36-char alphabet values)",
            "config": {"workload": workload, "baseline_config": args.config, "file_bytes": int(img.size),
                       "bytes_scanned_per_file": bytes_scanned, "entries_per_file": entries,
                       "io_type": "FileIO" if args.io == 0 else "Mmap",
                       "tuple_kind": "index16" if args.kind == 0 else "entry48",
                       "parallelism": f"one file per GPU x{world}"},
            "mentries_per_s": round(tot_entries / (t_max / args.steps) / 1e6, 2),
            "median_step": {"ms": round(med_ms, 4), "iters": med_iters,
                            "GiB_per_s_per_gpu": round(bytes_scanned / (med_ms * 1e-3) / 2**30, 3),
                            "method": "median of per-scan HIP event pairs on the scan stream (SURVEY.md 8(d)), "
                                      "after the wall-clock pass"},
            "hbm_read_frac_of_8TBs": round(tot_bytes / world / (t_max / args.steps) / 1e9 / PEAK_HBM_GBS, 4),
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": round(achieved, 1) if achieved else None,
                "peak": PEAK_HBM_GBS,
                "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBS, 4) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_kernel_ms": round(kms, 4),
                "avg_k_uniform_ms": round(run_ms, 4),
                "avg_k_sweep_ms": round(timed_scans.sweep_ms, 4),
                "avg_k_region_ms": round(main_ms, 4),
                "tail_phases_ms": timed_scans.phases,
                "run_entries": int(r.n_run),
                "avg_pipeline_ms": round(total_ms, 4),
                "algorithmic_bytes_per_launch": kbytes,
                # k_uniform also writes the run's tuples (16 or 48 B per entry, uni_post_fill / the verify
                # loop): read + written bytes over the same launch time, beside the read-only figure
                "achieved_incl_tuple_writes": (round((kbytes + int(r.n_run) * (16 if args.kind == 0 else 48))
                                                     / (kms * 1e-3) / 1e9, 1)
                                               if kname == "k_uniform" and kms > 0 else None),
                "practical_ceiling": {"kernel": "read-only reduction over the image (ldb_read_ceiling)",
                                      "GB_per_s": round(ceiling, 1) if ceiling else None,
                                      "frac": round(achieved / ceiling, 4) if achieved and ceiling else None},
            },
            "verified_vs_oracle": verified if world == 1 or all_ok is None else bool(all_ok == world),
            "status": int(r.status),
            "repairs": int(r.n_repairs),
            "fast_regions": int(r.n_fast),
            "regions": int(r.n_regions),
        }
        line["settle_steps"] = settle.last_steps
        line["host_enqueue_ms_per_step"] = round(timed_scans.enqueue_ms / args.steps, 4)
        if world > 1:
            line["roofline"]["per_rank"] = [
                {"rank": i, "kernel": kname, "avg_kernel_ms": round(v[1], 4),
                 "achieved": round(v[0] / (v[1] * 1e-3) / 1e9, 1) if v[1] > 0 else None,
                 "frac": round(v[0] / (v[1] * 1e-3) / 1e9 / PEAK_HBM_GBS, 4) if v[1] > 0 else None,
                 "avg_k_uniform_ms": round(v[2], 4), "avg_k_region_ms": round(v[3], 4),
                 "avg_pipeline_ms": round(v[4], 4), "wall_ms_per_step": round(v[5], 4)} for i, v in enumerate(per_rank)]
        if gather:
            line["gather"] = gather
        if e2e:
            line["e2e_host"] = e2e
        if legs:
            line["legs"] = legs
        if cpu:
            line["cpu_baseline"] = cpu
        print(json.dumps(line), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
