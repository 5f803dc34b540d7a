# A/B of k_uniform variants on one box: avg k_uniform ms (HIP events) per library variant, config 4.
set -o pipefail
mkdir -p gpurun_out
for v in liblazydb_gpu ${VARIANTS:-}; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python bench.py --config ${CFG:-4} --steps ${STEPS:-10} --warmup 2 --no-cpu --e2e 0 --legs= --pmc 0 --no-verify > gpurun_out/u_${v}.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/u_${v}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/u_${v}.log').read().strip().splitlines()[-1]); r=d['roofline']; print('${v}', 'k_uniform', r['avg_k_uniform_ms'], 'ms  pipeline', r['avg_pipeline_ms'], 'median', d['median_step']['ms'])"
done
