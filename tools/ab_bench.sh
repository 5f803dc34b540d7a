# A/B of library builds (tools/build_variants.py) on one box: each variant's bench line, alternating
# ROUNDS times so clock drift and box noise hit every variant alike.
# usage: VARIANTS="liblazydb_gpu var_x ..." ARGS="--config 4" ROUNDS=2 bash tools/ab_bench.sh TAG
set -o pipefail
TAG=${1:-ab}
mkdir -p gpurun_out
ARGS=${ARGS:-}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in ${VARIANTS:-liblazydb_gpu}; do
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu --e2e 0 \
      --legs= --pmc 0 $ARGS > gpurun_out/${TAG}_${v}_$r.json 2> gpurun_out/${TAG}_${v}_$r.err || { tail -5 gpurun_out/${TAG}_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/${TAG}_${v}_$r.json').read().strip().splitlines()[-1]); ro=d['roofline']
print('$v', 'round $r', d['value'], 'GiB/s', d['ms_per_step'], 'ms/step', 'median', d['median_step']['ms'], 'uni', ro['avg_k_uniform_ms'], 'sweep', ro.get('avg_k_sweep_ms'), 'region', ro.get('avg_k_region_ms', ro.get('avg_k_scan_main_ms')), 'pipe', ro['avg_pipeline_ms'], 'frac', ro['frac'], 'verified', d['verified_vs_oracle'])"
  done
done
