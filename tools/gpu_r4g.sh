set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4g_gputests.log 2>&1; rc=$?; tail -2 gpurun_out/r4g_gputests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r4g_gputests.log | head -30; exit $rc; }
LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_stamps.so timeout -k 10 200 python tools/uni_stamps.py || exit 1
VARIANTS="var_git_9d49948 liblazydb_gpu" CASES="w 3 1" ROUNDS=2 bash tools/scan_ab.sh || exit 1
T=r4g NOTEST=1 VARIANTS="var_git_9d49948 liblazydb_gpu var_def_LDB_UNI_FILLWAVE_0" ROUNDS=2 bash tools/gpu_session.sh
