# rocprofv3 evidence for the merge bench (config 5): kernel-trace stats, then FETCH/WRITE PMC passes
# on the merge kernels (one pass each, counters only).  usage: bash tools/profile_merge.sh <tag>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/profm_${1:-m}
mkdir -p $OUT
ARGS="--config 5 --steps 5 --warmup 1 --no-cpu --no-verify"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -f csv -- python3 bench.py $ARGS > $OUT/bench_under_kt.json 2> $OUT/kt.err || { tail -20 $OUT/kt.err; exit 1; }
i=0
for set in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-include-regex 'k_insert|k_live|k_emit_copy|k_scan_main|k_scan_write|k_uniform' -d $OUT/pmc$i -o pmc -f csv -- python3 bench.py $ARGS > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $OUT/pmc$i.log; exit 1; }
done
python3 tools/prof_summary.py $OUT > $OUT/summary.txt && cat $OUT/summary.txt
