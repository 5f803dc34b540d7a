# the default bench line (with every leg), then the N>1 paths rehearsed on this one-GPU box over gloo
set -o pipefail
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 - gpurun_out/${TAG}_bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("value", d["value"], "ms/step", d["ms_per_step"], "median", d["median_step"]["ms"], r["kernel"], r["avg_kernel_ms"], "frac", r["frac"], "traffic", r["traffic"], "verified", d["verified_vs_oracle"])
for l in d.get("legs", []):
    if l["config"] == 5:
        print(" leg 5", l["GiB_per_s"], l["phases_ms"], l["roofline"]["frac"], l["verified_vs_oracle"], l["cpu_baseline"])
    else:
        print(" leg", l["config"], l["GiB_per_s"], l["roofline_kernel"], l["roofline_frac"], "uni", l["k_uniform_ms"], "sweep", l.get("k_sweep_ms"), "region", l.get("k_region_ms"), l.get("tail_phases_ms"), "pipe", l["pipeline_ms"], "run", l["run_entries"], "/", l["entries"], "rerun", l["regions_rerun"], l["verified_vs_oracle"])
PY
LDB_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu --e2e 0 > gpurun_out/${TAG}_gloo2.json 2> gpurun_out/${TAG}_gloo2.err || { tail -20 gpurun_out/${TAG}_gloo2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_gloo2.json').read().strip().splitlines()[-1]);print('gloo2', d['value'], d['n_gpus'], d['verified_vs_oracle'], d.get('gather'))"
LDB_BENCH_BACKEND=gloo timeout -k 10 600 python bench.py --gpus 2 --config 5 --xmerge --xhash --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_xmerge2.json 2> gpurun_out/${TAG}_xmerge2.err || { tail -20 gpurun_out/${TAG}_xmerge2.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_xmerge2.json').read().strip().splitlines()[-1]);print('xmerge2', d['value'], d['n_gpus'], d['verified_vs_oracle'])"
