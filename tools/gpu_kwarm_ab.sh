# A/B of k_scan_main's chain warm-up (LDB_KWARM regions, default 2) on the GPU: the adversarial and
# region-pipeline GPU tests with each variant, the adversarial cases, then configs 3 and w.
set -o pipefail
mkdir -p gpurun_out
for v in var_def_LDB_KWARM_4 var_def_LDB_KWARM_8; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_adversarial.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/kw_$v.log 2>&1; rc=$?; tail -1 gpurun_out/kw_$v.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/kw_$v.log | head -30; exit $rc; }
done
for v in liblazydb_gpu var_def_LDB_KWARM_4 var_def_LDB_KWARM_8; do
  echo "== $v"
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 200 python tools/adversarial.py --cases embedded,mixed,binary --reps 3 || exit 1
done
VARIANTS="liblazydb_gpu var_def_LDB_KWARM_4 var_def_LDB_KWARM_8" CASES="3 w" ROUNDS=2 bash tools/scan_ab.sh || exit 1
