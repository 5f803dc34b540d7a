# GPU sweep: parity tests on the default library, then a short bench per library variant and
# config (CONFIGS, default "2"), one summary line each.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for c in ${CONFIGS:-2}; do
for v in liblazydb_gpu ${VARIANTS:-}; do
  LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/$v.so timeout -k 10 300 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu --e2e 0 --legs= --pmc 0 > gpurun_out/b_${v}_c$c.log 2>&1 || { echo "bench $v failed"; tail -5 gpurun_out/b_${v}_c$c.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/b_${v}_c$c.log').read().strip().splitlines()[-1]); print('cfg $c', '$v', d['value'], 'GiB/s', d['roofline']['avg_kernel_ms'], 'ms main', d['roofline']['avg_pipeline_ms'], 'ms total', 'verified', d['verified_vs_oracle'], 'repairs', d['repairs'])"
done
done
for st in stamps stamps1; do
  if [ -f lazydb_amd/_lib/var_$st.so ]; then
    LAZYDB_GPU_LIB=$PWD/lazydb_amd/_lib/var_$st.so timeout -k 10 200 python tools/stamps.py > gpurun_out/$st.log 2>&1 || { echo "$st failed"; tail -5 gpurun_out/$st.log; exit 1; }
    echo "== $st"; cat gpurun_out/$st.log
  fi
done
