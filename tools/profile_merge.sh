# rocprofv3 evidence for the config-5 merge: kernel-trace stats, then separate PMC passes (counters
# only, never combined with other traces) over the merge kernels.
# usage: bash tools/profile_merge.sh <tag>   -> gpurun_out/mprof_<tag>/...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r02}
OUT=gpurun_out/mprof_$TAG
mkdir -p $OUT
ARGS="--config 5 --no-cpu --no-verify --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -f csv -- python3 bench.py $ARGS > $OUT/bench_under_kt.json 2> $OUT/kt.err || { tail -20 $OUT/kt.err; exit 1; }
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE" "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-include-regex 'k_insert|k_live|k_emit_copy|k_uniform_batch' -d $OUT/pmc$i -o pmc -f csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
