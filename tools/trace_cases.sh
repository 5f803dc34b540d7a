# Kernel-trace stats of single workloads (tools/scan_one.py), one rocprofv3 run each, then optional
# PMC passes on k_scan_main at config 3.  usage: bash tools/trace_cases.sh <tag> [cases] [pmc]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-x}
CASES=${2:-"w 1 3"}
OUT=gpurun_out/tc_$TAG
mkdir -p $OUT
for c in $CASES; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/kt_$c -o kt -f csv -- python3 tools/scan_one.py $c 5 > $OUT/scan_$c.log 2>&1 || { tail -20 $OUT/scan_$c.log; exit 1; }
  tail -1 $OUT/scan_$c.log
  python3 - $OUT/kt_$c <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"   {r['Name'][:40]:40s} calls={r['Calls']:>5s} avg_ms={float(r['AverageNs'])/1e6:9.4f} tot_ms={float(r['TotalDurationNs'])/1e6:9.3f}")
PY
done
if [ -n "$3" ]; then
  KREGEX=k_scan_main BENCH_ARGS="--config 3 --legs= --pmc 0" bash tools/pmc_extra.sh $TAG
fi
