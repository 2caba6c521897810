# Bench-only variants (no parity: diagnostic builds produce wrong output on purpose).
# VARIANTS="name:ENV=val,..."
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in ${VARIANTS:-base:X=0}; do
  name=${v%%:*}; envs=${v#*:}
  env $(echo $envs | tr ',' ' ') timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab_$name.json 2>gpurun_out/ab_$name.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/ab_$name.json'));print('$name', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
