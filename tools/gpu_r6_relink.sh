# Round 6: the weak-chain ranking and the relink of runs passed over whole -- the GPU suite, then configs 3 / w
# and the 32 MiB 64-KiB-value writer mix for this build and a baseline, alternating (usage: TAG BASE)
set -o pipefail
TAG=${1:-relink}
BASE=${2:-var_git_073d431}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_gputests.txt 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_gputests.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in liblazydb_gpu $BASE; do
    echo "== $v round $r"
    for c in 3 w; do LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/scan_one.py $c 10 || exit 1; done
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 120 python tools/writer64k.py 64 || exit 1
  done
done
