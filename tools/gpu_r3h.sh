set -o pipefail
MB_ONLY=nost_LD_GATHER_CR_LP2_w16_db0_g1 timeout -k 10 200 ./tools/microbench/mb_uni 2>&1 | tail -1
VARIANTS="$(cd lazydb_amd/_lib && ls var_*.so | sed 's/\.so$//' | tr '\n' ' ')" bash tools/sweep_uni.sh
