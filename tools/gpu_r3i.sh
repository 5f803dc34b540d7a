set -o pipefail
MB_ONLY=nost_LD_GATHER_CR_LP2_w16_db0_g1 timeout -k 10 200 ./tools/microbench/mb_uni 2>&1 | tail -1
bash tools/sweep_uni.sh
CFG=2 bash tools/sweep_uni.sh
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_abi_contract.py > gpurun_out/r3i_tests.log 2>&1; tail -2 gpurun_out/r3i_tests.log
