# (var_def_LDB_FIN_ABL_8: built from a checkout of b0eb7f1, the last commit with the LDB_FIN_ABL switch)
set -o pipefail
timeout -k 10 300 python -u tools/sweep_check.py 64 > gpurun_out/sc.log 2>&1
for lib in lazydb_amd/_lib/liblazydb_gpu.so lazydb_amd/_lib/var_def_LDB_FIN_ABL_8.so; do
  LAZYDB_GPU_LIB=$PWD/$lib timeout -k 10 300 python -u tools/sweep_time.py 8192 10 || exit 1
done
MIB=1024 bash tools/gpu_sweep_abl.sh
