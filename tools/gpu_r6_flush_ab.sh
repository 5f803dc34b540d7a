# Round 6: the sweep's decode blocks software-pipelined -- sweep tests, then configs 3 / w, the 64K writer and
# the adversarial binary case, this build against a baseline, alternating (usage: TAG BASE)
set -o pipefail
TAG=${1:-flush}
BASE=${2:-var_git_HEAD}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep.py tests/test_gpu_parity.py tests/test_gpu_adversarial.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in liblazydb_gpu $BASE; do
    echo "== $v round $r"
    for c in 3 w; do LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/scan_one.py $c 10 || exit 1; done
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/writer64k.py 256 || exit 1
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 200 python tools/adversarial.py --mib 256 --cases binary,big,txlog > gpurun_out/${TAG}_adv_${v}_$r.jsonl || exit 1
    python3 -c "
import json
for l in open('gpurun_out/${TAG}_adv_${v}_$r.jsonl'):
    d = json.loads(l); print(d['case'], d['GiB_per_s'], 'sweep', d['k_sweep_ms'], 'region', d['k_region_ms'], 'n_sweep', d['n_sweep'])"
  done
done
