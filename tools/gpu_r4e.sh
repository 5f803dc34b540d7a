set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "piecewise or config1 or run_prefix or golden" > gpurun_out/r4e_focus.log 2>&1; rc=$?; tail -3 gpurun_out/r4e_focus.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r4e_focus.log | head -30; exit $rc; }
T=r4e VARIANTS="liblazydb_gpu" ROUNDS=1 bash tools/gpu_session.sh || exit 1
VARIANTS="liblazydb_gpu" CASES="1 3 w" ROUNDS=1 bash tools/scan_ab.sh
