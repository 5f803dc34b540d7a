set -o pipefail
mkdir -p gpurun_out
LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_stamps.so timeout -k 10 200 python tools/uni_stamps.py || exit 1
T=r4f NOTEST=1 VARIANTS="var_git_9d49948 liblazydb_gpu" ROUNDS=2 bash tools/gpu_session.sh || exit 1
VARIANTS="var_git_9d49948 liblazydb_gpu" CASES="1" ROUNDS=2 bash tools/scan_ab.sh
