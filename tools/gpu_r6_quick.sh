# Quick GPU check of the library: the sweep and parity test modules with a per-test timeout, then single
# workloads (tools/scan_one.py), each step under its own time limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_sweep.py} -m gpu -x -v --timeout 90 --timeout-method thread > gpurun_out/${1}_tests.txt 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Timeout|passed|failed" gpurun_out/${1}_tests.txt | tail -30; [ $rc -eq 0 ] || exit $rc
for c in ${2:-3 w 4 2}; do timeout -k 10 100 python -u tools/scan_one.py $c 10 || exit 1; done
