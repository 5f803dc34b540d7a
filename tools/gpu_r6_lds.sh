# Round 6: LDS tables below 64 KiB (k_uniform, k_sweep) -- the GPU suite, then bench lines for configs 4 / 2 and
# single-workload timings of configs 3 / w, this build against a baseline, alternating (usage: TAG BASE)
set -o pipefail
TAG=${1:-lds}
BASE=${2:-var_git_e52b845}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gputests.txt; [ $rc -eq 0 ] || exit $rc
VARIANTS="liblazydb_gpu $BASE" ARGS="--config 4" ROUNDS=2 bash tools/ab_bench.sh ${TAG}_c4 || exit 1
VARIANTS="liblazydb_gpu $BASE" ARGS="--config 2" ROUNDS=2 bash tools/ab_bench.sh ${TAG}_c2 || exit 1
for r in 1 2; do
  for v in liblazydb_gpu $BASE; do
    echo "== $v round $r"
    for c in 3 w; do LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/scan_one.py $c 10 || exit 1; done
  done
done
