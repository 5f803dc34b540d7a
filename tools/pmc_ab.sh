# PMC A/B of library variants on one box: one --pmc pass per variant over a short bench run.
# usage: VARIANTS="var_a var_b" bash tools/pmc_ab.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-ab}
CNT="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for v in ${VARIANTS}; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 rocprofv3 --pmc $CNT --kernel-include-regex 'k_scan_main' -d gpurun_out/pmcab_$TAG/$v -o pmc -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-verify --e2e 0 > gpurun_out/pmcab_${TAG}_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pmcab_${TAG}_$v.log; exit 1; }
done
