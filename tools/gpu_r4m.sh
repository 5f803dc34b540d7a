set -o pipefail
for c in 3 w; do LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_stamps.so timeout -k 10 200 python tools/stamps.py $c || exit 1; done
bash tools/pmc_scan.sh 3 r4 > gpurun_out/r4_pmc_cfg3.txt 2>&1 || exit 1
bash tools/pmc_scan.sh w r4 > gpurun_out/r4_pmc_w.txt 2>&1 || exit 1
cat gpurun_out/r4_pmc_cfg3.txt gpurun_out/r4_pmc_w.txt
