set -o pipefail
LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_stamps.so timeout -k 10 200 python tools/uni_stamps.py || exit 1
