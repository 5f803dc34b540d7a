set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bn
for n in 1 2 5; do
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/bn/kt$n -o kt -f csv -- python3 tools/batch_tier.py 512 $n w > gpurun_out/bn/run$n.txt 2> gpurun_out/bn/err$n.txt || { tail -5 gpurun_out/bn/err$n.txt; exit 1; }
cat gpurun_out/bn/run$n.txt
done
