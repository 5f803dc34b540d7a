# batched grid spread: GPU suite, then merge bench A/B (LDB_BATCH_SPREAD=0 / 1) and a verified run
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sp_gputests.txt 2>&1
rc=$?; tail -3 gpurun_out/sp_gputests.txt; [ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  LDB_BATCH_SPREAD=$v timeout -k 10 300 python bench.py --config 5 --steps 10 --no-cpu --no-verify > gpurun_out/sp_m$v.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/sp_m$v.json'));print('spread=$v',d['value'],d['ms_per_step'],d.get('phases_ms'))"
done
timeout -k 10 300 python bench.py --config 5 --steps 3 --no-cpu > gpurun_out/sp_mv.json && python3 -c "import json;d=json.load(open('gpurun_out/sp_mv.json'));print('verified',d['verified_vs_oracle'])" || exit 1
bash tools/kt_merge.sh sp
