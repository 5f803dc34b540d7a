# Sweep-tier A/B on both value kinds (Zipf text values, writer binary values): the product library and
# the var_*.so builds in lazydb_amd/_lib, alternating, 1 GiB each (MIB to change)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/kinds_ab.log
for rep in 1 2; do
  for kind in zipf writer; do
    for lib in lazydb_amd/_lib/liblazydb_gpu.so lazydb_amd/_lib/var_*.so; do
      [ -f "$lib" ] || continue
      echo -n "$kind " >> gpurun_out/kinds_ab.log
      LAZYDB_GPU_LIB=$PWD/$lib timeout -k 10 200 python -u tools/sweep_time.py ${MIB:-1024} 20 $kind 2>&1 | grep -v amdgpu.ids >> gpurun_out/kinds_ab.log || { tail -5 gpurun_out/kinds_ab.log; exit 1; }
    done
  done
done
cat gpurun_out/kinds_ab.log
