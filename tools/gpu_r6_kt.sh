# Kernel-trace stats of single workloads per library build (one box): usage bash tools/gpu_r6_kt.sh TAG "<libs>" "<cases>"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for v in $2; do
  for c in $3; do
    rm -rf gpurun_out/kt_${1}_${v}_$c
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_${1}_${v}_$c -o kt -f csv -- python3 tools/scan_one.py $c 20 > /dev/null 2>&1 || exit 1
    f=$(find gpurun_out/kt_${1}_${v}_$c -name "*kernel_stats.csv" | head -1)
    echo "== $v $c"; python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
    n=r['Name'][:60]
    if any(k in n for k in ('k_','uniform')): print('  %-60s calls %5s avg_us %9.1f' % (n, r['Calls'], float(r['AverageNs'])/1e3))
"
  done
done
