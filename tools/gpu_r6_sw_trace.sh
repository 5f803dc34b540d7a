# per-workgroup k_sweep trace (tools/sw_trace.py) of the writer batch: one by one, one launch, one launch per file
set -o pipefail
L=$PWD/lazydb_amd/_lib/var_def_LDB_SW_TRACE_1.so
LAZYDB_GPU_LIB=$L timeout -k 10 200 python tools/sw_trace.py single || exit 1
LDB_DEBUG=1 LDB_SWEEP_SPLIT=0 LAZYDB_GPU_LIB=$L timeout -k 10 200 python tools/sw_trace.py batch || exit 1
LDB_DEBUG=1 LDB_SWEEP_SPLIT=1 LAZYDB_GPU_LIB=$L timeout -k 10 200 python tools/sw_trace.py batch || exit 1
