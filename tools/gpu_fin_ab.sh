# k_sweep_fin A/B at 8 GiB (config 3's mix): the product library and the var_*.so builds in lazydb_amd/_lib
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/fin_ab.log
for rep in 1 2; do
  for lib in lazydb_amd/_lib/liblazydb_gpu.so lazydb_amd/_lib/var_*.so; do
    [ -f "$lib" ] || continue
    LAZYDB_GPU_LIB=$PWD/$lib timeout -k 10 200 python -u tools/sweep_time.py ${MIB:-8192} 10 >> gpurun_out/fin_ab.log 2>&1 || { tail -5 gpurun_out/fin_ab.log; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/fin_ab.log
