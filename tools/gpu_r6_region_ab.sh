# Round 6: the region pipeline alone (LDB_SWEEP=0) in this build's k_region against round 5's separate kernels
# (a git build), on the adversarial logs, alternating (usage: TAG BASE)
set -o pipefail
TAG=${1:-region}
BASE=${2:-var_git_0a1256e}
mkdir -p gpurun_out
for r in 1 2; do
  for v in liblazydb_gpu $BASE; do
    echo "== $v round $r"
    LDB_DEBUG=1 LDB_SWEEP=0 LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python tools/adversarial.py --mib 256 --cases txlog,mixed,binary,big > gpurun_out/${TAG}_adv_${v}_$r.jsonl || exit 1
    python3 -c "
import json
for l in open('gpurun_out/${TAG}_adv_${v}_$r.jsonl'):
    d = json.loads(l); print(d['case'], d['GiB_per_s'], 'ms', d['ms'], 'n_regions', d['n_regions'], 'n_sweep', d['n_sweep'], 'pipe', d.get('pipeline_ms'))"
  done
done
