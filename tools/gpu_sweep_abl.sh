# The sweep tier's attribution on one box: the product library and the LDB_SW_ABL builds present in
# lazydb_amd/_lib (tools/build_variants.py def_LDB_SW_ABL=<bits> on a checkout of b0eb7f1), on a 1 GiB Zipf log; then the read ceiling.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/abl.log
for lib in lazydb_amd/_lib/liblazydb_gpu.so lazydb_amd/_lib/var_*.so lazydb_amd/_lib/liblazydb_gpu.so; do
  [ -f "$lib" ] || continue
  LAZYDB_GPU_LIB=$PWD/$lib timeout -k 10 120 python -u tools/sweep_time.py ${MIB:-1024} 20 >> gpurun_out/abl.log 2>&1 || { tail -5 gpurun_out/abl.log; exit 1; }
done
grep -v amdgpu.ids gpurun_out/abl.log
