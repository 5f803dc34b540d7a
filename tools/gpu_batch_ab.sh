# merge: parity tests, the bench (verified) and a kernel trace
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_merge.py tests/test_gpu_xmerge.py > gpurun_out/r2e_tests.log 2>&1 || { tail -30 gpurun_out/r2e_tests.log; exit 1; }
tail -2 gpurun_out/r2e_tests.log
timeout -k 10 300 python bench.py --config 5 --steps 10 --no-cpu --no-verify > gpurun_out/r2e_merge.json || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/r2e_merge.json'));print(d['value'],d['ms_per_step'],d['phases_ms'])"
timeout -k 10 300 python bench.py --config 5 --steps 3 --no-cpu > gpurun_out/r2e_merge_verify.json && python3 -c "import json;d=json.load(open('gpurun_out/r2e_merge_verify.json'));print('verified',d['verified_vs_oracle'])"
bash tools/kt_merge.sh ${1:-e}
