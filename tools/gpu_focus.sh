# The run prefix's focus check on one box: the piecewise-run / config-1 / run-prefix GPU tests, the
# k_uniform phase stamps (tools/uni_stamps.py, var_stamps.so), config 1 A/B of liblazydb_gpu against V2,
# and with BENCH=1 the main bench line A/B (tools/gpu_session.sh).
# usage: V2=var_x [BENCH=1] bash tools/gpu_focus.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "piecewise or config1 or run_prefix" > gpurun_out/focus.log 2>&1; rc=$?; tail -2 gpurun_out/focus.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/focus.log | head -30; exit $rc; }
LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_stamps.so timeout -k 10 200 python tools/uni_stamps.py || exit 1
VARIANTS="liblazydb_gpu ${V2:-}" CASES="1" ROUNDS=2 bash tools/scan_ab.sh || exit 1
[ -z "$BENCH" ] || T=focus NOTEST=1 VARIANTS="liblazydb_gpu ${V2:-}" ROUNDS=2 bash tools/gpu_session.sh
