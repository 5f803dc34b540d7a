# k_scan_main on config 3 and the writer mix: phase stamps (var_stamps.so), PMC passes (tools/pmc_scan.sh)
# and the instruction-cache counters. usage: bash tools/gpu_scan_profile.sh <tag>
set -o pipefail
T=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in 3 w; do LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_stamps.so timeout -k 10 200 python tools/stamps.py $c || exit 1; done
bash tools/pmc_scan.sh 3 $T > gpurun_out/${T}_pmc_cfg3.txt 2>&1 || exit 1
bash tools/pmc_scan.sh w $T > gpurun_out/${T}_pmc_w.txt 2>&1 || exit 1
for c in 3 w; do
  OUT=gpurun_out/pmci_${T}_$c; mkdir -p $OUT
  timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_IFETCH --kernel-include-regex k_scan_main -d $OUT/p1 -o pmc -f csv -- python3 tools/scan_one.py $c 3 > $OUT/p1.log 2>&1 || { echo "icache pass failed"; exit 1; }
done
cat gpurun_out/${T}_pmc_cfg3.txt gpurun_out/${T}_pmc_w.txt
