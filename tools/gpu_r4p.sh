set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4p_gputests.log 2>&1; rc=$?; tail -2 gpurun_out/r4p_gputests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r4p_gputests.log | head -30; exit $rc; }
VARIANTS="liblazydb_gpu var_git_9d49948" CASES="3 w" ROUNDS=2 bash tools/scan_ab.sh || exit 1
timeout -k 10 400 python tools/adversarial.py > gpurun_out/r04p_adv.jsonl 2>gpurun_out/r04p_adv.err || exit 1
cat gpurun_out/r04p_adv.jsonl
