# For each VARIANTS entry "name:ENV=val,...": quick parity subset + bench (no profiler).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in ${VARIANTS:-base:X=0}; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "config2 or config3 or acquire or prioritized or limiter or param" > gpurun_out/par_$name.log 2>&1
  rc=$?; echo "$name parity: $(tail -1 gpurun_out/par_$name.log)"; [ $rc -eq 0 ] || exit $rc
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$name.json 2>gpurun_out/ab_$name.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print('$name', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
