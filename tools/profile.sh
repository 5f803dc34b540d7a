# rocprofv3 evidence for the bench: kernel-trace stats of the default bench command, then separate
# PMC passes (counters only, never combined with other traces) on a short bench run.
# usage: bash tools/profile.sh <tag>   -> gpurun_out/prof_<tag>/...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH_ARGS=${BENCH_ARGS:-}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -f csv -- python3 bench.py --legs= --pmc 0 $BENCH_ARGS > $OUT/bench_under_kt.json 2> $OUT/kt.err || { tail -20 $OUT/kt.err; exit 1; }
tail -1 $OUT/bench_under_kt.json
SHORT="--steps 5 --warmup 1 --no-cpu --no-verify --legs= --e2e 0 --pmc 0"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
           "SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-include-regex 'k_uniform|k_sweep|k_region' -d $OUT/pmc$i -o pmc -f csv -- python3 bench.py $SHORT > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
python3 tools/prof_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
