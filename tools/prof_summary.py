"""Summarise a tools/profile.sh output directory: kernel-trace stats + per-dispatch PMC averages.

FETCH_SIZE is doubled (gfx950 reports half the bytes of wide coalesced streaming reads,
MI355X_MICROARCH.md "HBM"); SQ_*CYCLES count quad-cycles.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    for k, v in (("k_uniform_fill", "k_uniform_fill"), ("k_uniform_batch", "k_uniform_batch"),
                 ("k_uniform<true", "k_uniform_chunk"), ("k_uniform<false, true>", "k_uniform_hash")):
        if k in name:
            return v
    for k in ("k_uniform", "k_sweep", "k_region", "k_init", "k_batch_init", "k_serial", "k_fallback",
              "k_locate", "k_insert", "k_live", "k_scan_reduce", "k_scan_tiles", "k_scan_write", "k_pack",
              "k_emit_copy"):
        if k in name:
            return k
    return name[:60]


def main(d: str) -> None:
    for f in glob.glob(os.path.join(d, "kt", "**", "*kernel_stats.csv"), recursive=True):
        print(f"== kernel stats ({os.path.relpath(f, d)})")
        with open(f) as fh:
            rows = list(csv.DictReader(fh))
        for r in rows:
            print(f"{short(r['Name']):16s} calls={r['Calls']:>6s} avg_ms={float(r['AverageNs']) / 1e6:9.4f} "
                  f"min_ms={float(r['MinNs']) / 1e6:9.4f} max_ms={float(r['MaxNs']) / 1e6:9.4f} pct={float(r['Percentage']):6.2f}")
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                key = (r.get("Dispatch_Id") or r.get("Dispatch_ID") or r.get("Correlation_Id"), r["Counter_Name"])
                acc[short(r["Kernel_Name"])][key].append(float(r["Counter_Value"]))
    pmc = {}
    for k, m in acc.items():
        per = defaultdict(list)
        for (disp, cname), vals in m.items():
            per[cname].append(sum(vals))
        print(f"== PMC {k} (per dispatch averages over {max(len(v) for v in per.values())} dispatches)")
        for cname in sorted(per):
            v = sum(per[cname]) / len(per[cname])
            extra = ""
            if cname == "FETCH_SIZE":
                extra = f"  -> corrected x2 = {2 * v * 1024 / 1e6:.1f} MB (FETCH_SIZE unit KiB)"
            if cname == "WRITE_SIZE":
                extra = f"  -> {v * 1024 / 1e6:.1f} MB"
            print(f"  {cname:24s} {v:16.1f}{extra}")
            pmc.setdefault(k, {})[cname] = v
    for k in ("k_uniform", "k_sweep", "k_region"):
        if k in pmc and "FETCH_SIZE" in pmc[k]:
            pmc[k]["hbm_read_bytes_per_launch"] = pmc[k]["FETCH_SIZE"] * 2 * 1024
    with open(os.path.join(d, "pmc.json"), "w") as f:
        json.dump(pmc, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(sys.argv[1])
