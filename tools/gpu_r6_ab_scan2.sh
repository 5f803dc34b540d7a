# single-workload A/B of library builds (configs 3 / w and the writer-64K log), alternating
# usage: VARIANTS="liblazydb_gpu var_x" bash tools/gpu_r6_ab_scan2.sh TAG
set -o pipefail
for r in 1 2; do
  for v in ${VARIANTS:-liblazydb_gpu}; do
    echo "== $v round $r"
    for c in 3 w; do LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/scan_one.py $c 10 || exit 1; done
  done
done
