# config 3 only (tools/scan_one.py), VARIANTS alternating for ROUNDS rounds
set -o pipefail
for r in $(seq 1 ${ROUNDS:-4}); do
  for v in ${VARIANTS:-liblazydb_gpu}; do
    echo "== $v round $r"
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/scan_one.py 3 10 || exit 1
  done
done
