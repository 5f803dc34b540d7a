# Round 6: the GPU suite, then single-workload timings (tools/scan_one.py) and an A/B of bench lines against
# a baseline build (usage: bash tools/gpu_r6_check.sh TAG [baseline_lib_name] [cases])
set -o pipefail
TAG=${1:-x}
BASE=${2:-}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.txt 2>&1
rc=$?; tail -15 gpurun_out/${TAG}_gputests.txt; [ $rc -eq 0 ] || exit $rc
for c in ${3:-4 2 3 w}; do timeout -k 10 120 python tools/scan_one.py $c 10 || exit 1; done
if [ -n "$BASE" ]; then
  VARIANTS="liblazydb_gpu $BASE" ARGS="--config 4" ROUNDS=2 bash tools/ab_bench.sh ${TAG}_c4 || exit 1
  VARIANTS="liblazydb_gpu $BASE" ARGS="--config 2" ROUNDS=2 bash tools/ab_bench.sh ${TAG}_c2 || exit 1
fi
