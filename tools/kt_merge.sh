# kernel trace of the merge bench (config 5): bash tools/kt_merge.sh <tag>  (stats + per-dispatch trace)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ktm_${1:-m}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -f csv -- python3 bench.py --config 5 --steps 5 --warmup 1 --no-cpu --no-verify > $OUT/bench.json 2> $OUT/kt.err || { tail -20 $OUT/kt.err; exit 1; }
python3 tools/prof_summary.py $OUT | head -30
