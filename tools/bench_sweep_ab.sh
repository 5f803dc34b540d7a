set -o pipefail
mkdir -p gpurun_out
for sw in 1 0 1 0; do
  LDB_SWEEP=$sw timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --e2e 0 --pmc 0 --legs 2,3,w --no-verify > gpurun_out/bsw_$sw.json 2> gpurun_out/bsw_$sw.err || { tail -5 gpurun_out/bsw_$sw.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/bsw_$sw.json').read().strip().splitlines()[-1])
print('sweep=$sw', 'cfg4 ms', d['ms_per_step'], 'median', d['median_step']['ms'], 'pipe', d['roofline']['avg_pipeline_ms'])
for l in d['legs']: print('   leg', l['config'], 'ms', l['ms_per_step'], 'median', l['median_event_ms'], 'pipe', l['pipeline_ms'], 'sweep', l.get('k_sweep_ms'), 'region', l.get('k_region_ms'), l.get('tail_phases_ms'), 'n_sweep', l.get('sweep_entries'))
"
done
