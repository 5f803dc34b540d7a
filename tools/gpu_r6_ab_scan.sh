# Same-box A/B of single workloads (tools/scan_one.py) between library builds, alternating.
# usage: bash tools/gpu_r6_ab_scan.sh "<lib names>" "<cases>" [rounds]
set -o pipefail
for r in $(seq 1 ${3:-2}); do
  for v in $1; do
    for c in $2; do
      echo -n "$v r$r: "
      LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/scan_one.py $c 20 || exit 1
    done
  done
done
