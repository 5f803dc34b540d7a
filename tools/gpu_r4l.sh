set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4l_gputests.log 2>&1; rc=$?; tail -2 gpurun_out/r4l_gputests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r4l_gputests.log | head -30; exit $rc; }
VARIANTS="liblazydb_gpu var_def_LDB_ST_NT_1 var_git_9d49948" CASES="3 w" ROUNDS=2 bash tools/scan_ab.sh || exit 1
