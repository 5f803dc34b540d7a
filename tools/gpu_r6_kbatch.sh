# Round 6: batch pipes by value in the kernel arguments (global, not flat, accesses in k_sweep<true> /
# k_region<true>): batch tests, the one-launch / per-file sweep A/B, then the per-workgroup trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_binding.py tests/test_gpu_merge.py tests/test_gpu_sweep.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/kb_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/kb_tests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    echo "== LDB_SWEEP_SPLIT=$v round $r"
    LDB_DEBUG=1 LDB_SWEEP_SPLIT=$v timeout -k 10 300 python tools/batch_tier.py 512 || exit 1
    LDB_DEBUG=1 LDB_SWEEP_SPLIT=$v timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu --e2e 0 --legs= --pmc 0 > gpurun_out/kb_m_${v}_${r}.json 2> gpurun_out/kb_m_${v}_${r}.err || { tail -5 gpurun_out/kb_m_${v}_${r}.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/kb_m_${v}_${r}.json').read().strip().splitlines()[-1])
print('merge', d['value'], d['unit'], d['ms_per_step'], 'ms', d.get('phases_ms'), 'verified', d.get('verified_vs_oracle'))"
  done
done
L=$PWD/lazydb_amd/_lib/var_def_LDB_SW_TRACE_1.so
LDB_DEBUG=1 LDB_SWEEP_SPLIT=0 LAZYDB_GPU_LIB=$L timeout -k 10 200 python tools/sw_trace.py batch || exit 1
