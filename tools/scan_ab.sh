# A/B of library builds on single workloads (tools/scan_one.py), alternating ROUNDS times.
# usage: VARIANTS="liblazydb_gpu var_x" CASES="3 w 1" ROUNDS=2 bash tools/scan_ab.sh
set -o pipefail
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in ${CASES:-3}; do
    for v in ${VARIANTS:-liblazydb_gpu}; do
      echo -n "$v r$r "
      LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 200 python tools/scan_one.py $c ${REPS:-10} || exit 1
    done
  done
done
