# Round-5 profiles of config 3 (8 GiB Zipf log, the sweep tier): kernel-trace stats of bench.py --config 3,
# then PMC passes on k_sweep / k_sweep_fin (tools/pmc_sweep.sh at 8 GiB). Outputs under gpurun_out/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r05_cfg3
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_cfg3/kt -o kt -f csv -- python3 bench.py --config 3 --steps 20 --warmup 5 --no-cpu --e2e 0 --pmc 0 --legs "" > gpurun_out/r05_cfg3/bench.json 2> gpurun_out/r05_cfg3/bench.err || exit 1
MIB=8192 bash tools/pmc_sweep.sh r05cfg3 > gpurun_out/r05_cfg3/pmc_sweep.txt 2>&1 || exit 1
