# Parity tests + bench variants (no profiler).  VARIANTS="name:ENV=val,ENV2=val ..."
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; grep -E "Error|assert " gpurun_out/gpu_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-base:X=0}; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab_$name.json 2>gpurun_out/ab_$name.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print('$name', d['value'], d['roofline']['kernel'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
