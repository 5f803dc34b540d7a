# GPU check at HEAD: parity tests of the scan path, then a short bench line (config 4 + legs).
# usage: bash tools/gpu_check.sh TAG [pytest selection...]
set -o pipefail
TAG=${1:-x}; shift
SEL=${@:-tests/test_gpu_parity.py tests/test_gpu_abi_contract.py}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread $SEL > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_tests.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --no-cpu --e2e 0 --legs ${LEGS:-2,3} --pmc 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "median", d.get("median_step", {}).get("ms"), "kernel", r["kernel"], r["avg_kernel_ms"], "frac", r["frac"], "pipeline", r["avg_pipeline_ms"], "verified", d["verified_vs_oracle"])
for l in d.get("legs", []):
    print(" leg", l["config"], l["GiB_per_s"], "GiB/s", l["roofline_kernel"], l["roofline_frac"], "uni", l["k_uniform_ms"], "main", l["k_scan_main_ms"], "pipe", l["pipeline_ms"], "verified", l["verified_vs_oracle"])
PY
