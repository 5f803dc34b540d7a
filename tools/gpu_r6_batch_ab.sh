# Round 6: the batched k_sweep (an item loop over a CU-sized grid) -- batch tests, then the batched tier
# (tools/batch_tier.py) and the config-5 merge for this build and a baseline, alternating (usage: TAG BASE)
set -o pipefail
TAG=${1:-batch}
BASE=${2:-var_git_HEAD}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_binding.py tests/test_gpu_merge.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in liblazydb_gpu $BASE; do
    echo "== $v round $r"
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python tools/batch_tier.py 512 || exit 1
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu --e2e 0 --legs= --pmc 0 > gpurun_out/${TAG}_m_${v}_$r.json 2> gpurun_out/${TAG}_m_${v}_$r.err || { tail -5 gpurun_out/${TAG}_m_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_m_${v}_$r.json').read().strip().splitlines()[-1])
print('merge', d['value'], d['unit'], d['ms_per_step'], 'ms', d.get('phases_ms'), 'verified', d.get('verified_vs_oracle'))"
  done
done
