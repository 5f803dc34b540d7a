set -o pipefail
mkdir -p gpurun_out
LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_def_LDB_FOLD_INIT_1.so timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4u_gputests.log 2>&1; rc=$?; tail -2 gpurun_out/r4u_gputests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r4u_gputests.log | head -30; exit $rc; }
VARIANTS="liblazydb_gpu var_def_LDB_FOLD_INIT_1" CASES="1" ROUNDS=2 bash tools/scan_ab.sh || exit 1
T=r4u NOTEST=1 VARIANTS="var_def_LDB_FOLD_INIT_1 liblazydb_gpu" ROUNDS=2 bash tools/gpu_session.sh
