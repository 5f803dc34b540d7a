# GPU A/B sweep: parity tests on the default library, then per library variant and config a short
# bench line, then the stamps phase breakdown (LDB_STAMPS build) of the given configs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for c in ${CONFIGS:-2}; do
for v in liblazydb_gpu ${VARIANTS:-}; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu --e2e 0 --legs= --pmc 0 ${NOVERIFY:+--no-verify} > gpurun_out/b_${v}_c$c.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/b_${v}_c$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_${v}_c$c.log').read().strip().splitlines()[-1]); print('cfg $c', '$v', d['value'], 'GiB/s', d['roofline']['avg_kernel_ms'], 'ms main', d['roofline']['avg_pipeline_ms'], 'ms total', 'verified', d['verified_vs_oracle'], 'fast', d['fast_regions'], '/', d['regions'])"
done
done
for c in ${STAMP_CONFIGS:-}; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_stamps.so timeout -k 10 200 python tools/stamps.py $c > gpurun_out/stamps_c$c.log 2>&1 || { echo "stamps failed"; tail -5 gpurun_out/stamps_c$c.log; exit 1; }
  echo "== stamps cfg $c"; cat gpurun_out/stamps_c$c.log
done
