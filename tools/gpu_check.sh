# GPU suite, single-workload timings and the adversarial suite (one gpurun call).
# usage: bash tools/gpu_check.sh <tag> [cases for scan_one]
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gputests.txt; [ $rc -eq 0 ] || exit $rc
for c in ${2:-w 1 3 2}; do timeout -k 10 120 python tools/scan_one.py $c 10 || exit 1; done
timeout -k 10 300 python tools/adversarial.py --mib 256 --reps 3 > gpurun_out/${TAG}_adv.jsonl 2>gpurun_out/${TAG}_adv.err || exit 1
python3 -c "
import json
for l in open('gpurun_out/${TAG}_adv.jsonl'):
    d=json.loads(l); print(d['case'], d['GiB_per_s'], 'GiB/s', d['pipeline_ms'], 'ms repairs', d['n_repairs'], 'broken', d['n_broken_after_walk'], 'fast', d['n_fast'], '/', d['n_regions'], d['verified'])
"
