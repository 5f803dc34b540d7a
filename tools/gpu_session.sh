# One GPU session: the -m gpu suite, then an A/B of library variants on the main bench line.
# usage: T=tag VARIANTS="..." ROUNDS=n [ARGS=...] [NOTEST=1] bash tools/gpu_session.sh
set -o pipefail
mkdir -p gpurun_out
T=${T:-s}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1; rc=$?
  tail -2 gpurun_out/${T}_gputests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${T}_gputests.log | head -20; exit $rc; }
fi
[ -z "$VARIANTS" ] || bash tools/ab_bench.sh ${T}_ab || exit 1
