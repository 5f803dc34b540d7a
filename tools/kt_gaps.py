"""Per-kernel durations and the gaps between them for the last pipelines of a rocprofv3 kernel trace.
usage: python tools/kt_gaps.py gpurun_out/<dir>/kt_kernel_trace.csv [first-kernel-name] [count]"""
import csv
import sys

KN = ('k_uniform_fill', 'k_uniform', 'k_scan_main', 'k_fallback', 'k_link', 'k_repair', 'k_combine', 'k_compact', 'k_serial')


def name(r):
    k = r['Kernel_Name']
    for c in KN:
        if c + '(' in k or c + '<' in k:
            return c
    return k[:40]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
first = sys.argv[2] if len(sys.argv) > 2 else 'k_uniform'
names = [name(r) for r in rows]
starts = [i for i, n in enumerate(names) if n == first]
for st in starts[-(int(sys.argv[3]) if len(sys.argv) > 3 else 2):]:
    t0, prev = int(rows[st]['Start_Timestamp']), None
    print('---')
    for r, n in zip(rows[st:st + 12], names[st:st + 12]):
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        print(f"{n:22s} start {(s - t0) / 1e3:8.1f} us  dur {(e - s) / 1e3:8.1f}  gap {((s - prev) / 1e3 if prev else 0):6.1f}")
        prev = e
