# Round 6 final check: the GPU suite, smoke(), and the default bench line, each under its own limit
set -o pipefail
T=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputests.txt 2>&1
rc=$?; tail -3 gpurun_out/${T}_gputests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['unit'], d['ms_per_step'], 'frac', d['roofline']['frac'], 'k_uniform', d['roofline']['avg_k_uniform_ms'])
for l in d['legs']: print(l['config'], l.get('GiB_per_s'), l.get('ms_per_step'))"
