# Adversarial logs (tools/adversarial.py, 256 MiB, verified) per library build on one box
set -o pipefail
mkdir -p gpurun_out
for v in $2; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python tools/adversarial.py --mib 256 --reps 3 > gpurun_out/${1}_${v}_adv.jsonl 2>gpurun_out/${1}_${v}_adv.err || { tail -5 gpurun_out/${1}_${v}_adv.err; exit 1; }
  python3 -c "
import json
for l in open('gpurun_out/${1}_${v}_adv.jsonl'):
    d=json.loads(l); print('$v', d['case'], d['GiB_per_s'], 'GiB/s', d['ms'], 'ms sweep', d.get('n_sweep'), 'fast', d['n_fast'], '/', d['n_regions'], 'rerun', d['n_repairs'], d['verified'])
"
done
