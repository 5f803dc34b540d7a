set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kt4
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt4 -o kt -- python3 bench.py --legs "" --no-cpu --steps 30 --warmup 5 --pmc 0 --e2e 0 --no-verify > gpurun_out/kt4/bench.log 2>&1
