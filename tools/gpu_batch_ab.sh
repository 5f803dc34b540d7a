# merge A/B: batched run-prefix grid (workgroups per CU) and the scan batch switch
set -o pipefail
mkdir -p gpurun_out
for V in "LDB_UNI_BATCH_BPC=2" "LDB_UNI_BATCH_BPC=4" "LDB_UNI_BATCH_BPC=8" "LDB_UNI_BATCH_BPC=1"; do env $V timeout -k 10 300 python bench.py --config 5 --steps 10 --no-cpu --no-verify > gpurun_out/r2c_merge_$V.json || exit 1; python3 -c "import json;d=json.load(open('gpurun_out/r2c_merge_$V.json'));print('$V',d['value'],d['ms_per_step'],d['phases_ms'])"; done
