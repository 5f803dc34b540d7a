# Full GPU evidence at HEAD: the -m gpu suite, smoke, the default bench line, then the rocprof profile.
# usage: bash tools/gpu_full.sh TAG
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_gputests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_gputests.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
tail -c 1500 gpurun_out/${TAG}_bench.json
[ -n "$NOPROF" ] || bash tools/profile.sh ${TAG}
