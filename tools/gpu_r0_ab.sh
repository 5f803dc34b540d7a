# A/B of round 0's probe count (LDB_UNI_R0) in the run search: run-prefix GPU tests with each variant, then config 1.
set -o pipefail
mkdir -p gpurun_out
for v in var_def_LDB_UNI_R0_1024 var_def_LDB_UNI_R0_512; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "piecewise or config1 or run_prefix" > gpurun_out/r0_$v.log 2>&1; rc=$?; tail -1 gpurun_out/r0_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r0_$v.log | head -30; exit $rc; }
done
VARIANTS="liblazydb_gpu var_def_LDB_UNI_R0_1024 var_def_LDB_UNI_R0_512" CASES="1" ROUNDS=3 bash tools/scan_ab.sh || exit 1
