# Round evidence: the default bench line, its rocprofv3 kernel-trace + PMC summaries, the merge's,
# and config 1's FETCH. usage: bash tools/gpu_evidence.sh <tag>
set -o pipefail
T=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 900 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
tail -c 600 gpurun_out/${T}_bench.json; echo
bash tools/profile.sh $T > gpurun_out/${T}_profile.log 2>&1 || { tail -20 gpurun_out/${T}_profile.log; exit 1; }
bash tools/profile_merge.sh $T > gpurun_out/${T}_mprofile.log 2>&1 || { tail -20 gpurun_out/${T}_mprofile.log; exit 1; }
KREGEX=k_uniform bash tools/pmc_scan.sh 1 $T > gpurun_out/${T}_pmc_cfg1.txt 2>&1 || { tail -20 gpurun_out/${T}_pmc_cfg1.txt; exit 1; }

# config 3 through the host API (PCIe-inclusive e2e leg) and the batched replay through the tier
timeout -k 10 600 python bench.py --config 3 --legs= --pmc 0 --no-cpu --steps 10 > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 1; }
timeout -k 10 600 python tools/batch_tier.py 1024 > gpurun_out/${T}_batch.txt 2>&1 || { tail -20 gpurun_out/${T}_batch.txt; exit 1; }
cat gpurun_out/${T}_batch.txt
echo done
