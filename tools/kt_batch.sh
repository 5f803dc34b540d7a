# kernel trace of the batched tier (tools/batch_tier.py, writer mix + Zipf batches): per-kernel stats
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/ktb_${1:-x}
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt -f csv -- python3 tools/batch_tier.py 512 > $OUT/run.txt 2> $OUT/kt.err || { tail -20 $OUT/kt.err; exit 1; }
cat $OUT/run.txt
python3 tools/prof_summary.py $OUT | head -20
