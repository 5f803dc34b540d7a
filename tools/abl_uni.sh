set -o pipefail
for v in liblazydb_gpu ${VARIANTS:-var_def_LDB_UNI_ABL_1 var_def_LDB_UNI_ABL_2}; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 200 python bench.py --config 4 --steps 30 --warmup 3 --no-cpu --no-verify --e2e 0 --legs= --pmc 0 > gpurun_out/abl_$v.log 2>&1 || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1]); print('$v', d['roofline']['avg_k_uniform_ms'], d['roofline']['run_entries'])"
done
