# kernel trace of the writer batch with LDB_SWEEP_SPLIT=1 (one k_sweep<false> launch per file)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/sk
LDB_DEBUG=1 LDB_SWEEP_SPLIT=1 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/sk/kt -o kt -f csv -- python3 tools/batch_tier.py 512 5 w > gpurun_out/sk/run.txt 2> gpurun_out/sk/err.txt || { tail -5 gpurun_out/sk/err.txt; exit 1; }
cat gpurun_out/sk/run.txt
