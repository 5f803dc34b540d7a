# Round 6: the sweep tier's stop word (run 0 ends the tier early) -- sweep tests, then adversarial cases and
# configs 3 / w for the current build and a baseline build, alternating (usage: bash tools/gpu_r6_stop.sh TAG BASE)
set -o pipefail
TAG=${1:-stop}
BASE=${2:-var_git_HEAD}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -5 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in liblazydb_gpu $BASE; do
    echo "== $v round $r"
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python tools/adversarial.py --mib 256 --cases mixed,embedded,binary,txlog > gpurun_out/${TAG}_adv_${v}_$r.jsonl || exit 1
    python3 -c "
import json
for l in open('gpurun_out/${TAG}_adv_${v}_$r.jsonl'):
    d = json.loads(l); print(d['case'], d['GiB_per_s'], 'sweep', d['k_sweep_ms'], 'region', d['k_region_ms'], 'n_sweep', d['n_sweep'])"
    for c in 3 w; do LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/scan_one.py $c 10 || exit 1; done
  done
done
