# Round 6: the batched sweep as one launch over (vg, n) against one k_sweep<true> launch per file
# (LDB_SWEEP_SPLIT=1), alternating; batch tests first
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_binding.py tests/test_gpu_merge.py -m gpu -x -q --timeout 300 --timeout-method thread -k batch > gpurun_out/split_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/split_tests.txt; [ $rc -eq 0 ] || exit $rc
LDB_DEBUG=1 LDB_SWEEP_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_binding.py tests/test_gpu_merge.py -m gpu -x -q --timeout 300 --timeout-method thread -k batch > gpurun_out/split_tests1.txt 2>&1
rc=$?; tail -2 gpurun_out/split_tests1.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    echo "== LDB_SWEEP_SPLIT=$v round $r"
    LDB_DEBUG=1 LDB_SWEEP_SPLIT=$v timeout -k 10 300 python tools/batch_tier.py 512 || exit 1
    LDB_DEBUG=1 LDB_SWEEP_SPLIT=$v timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu --e2e 0 --legs= --pmc 0 > gpurun_out/split_m_${v}_${r}.json 2> gpurun_out/split_m_${v}_${r}.err || { tail -5 gpurun_out/split_m_${v}_${r}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/split_m_${v}_${r}.json').read().strip().splitlines()[-1])
print('merge', d['value'], d['unit'], d['ms_per_step'], 'ms', d.get('phases_ms'), 'verified', d.get('verified_vs_oracle'))"
  done
done
