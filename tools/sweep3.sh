# GPU A/B timing only (no tests): a short bench line per library variant and config.
set -o pipefail
mkdir -p gpurun_out
for c in ${CONFIGS:-2}; do
for v in liblazydb_gpu ${VARIANTS:-}; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu --e2e 0 --legs= --pmc 0 ${NOVERIFY:+--no-verify} > gpurun_out/b_${v}_c$c.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/b_${v}_c$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_${v}_c$c.log').read().strip().splitlines()[-1]); print('cfg $c', '$v', d['value'], 'GiB/s', d['roofline']['kernel'], d['roofline']['avg_kernel_ms'], 'ms', d['roofline']['frac'], 'frac', d['roofline']['avg_pipeline_ms'], 'ms total', 'verified', d['verified_vs_oracle'], 'fast', d['fast_regions'], '/', d['regions'])"
done
done
