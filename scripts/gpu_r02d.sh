# Param paths (slot vs per-rule walk), shared sketch (per-level launches / cooperative), flow bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02d}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_param_rules_gpu.py tests/test_param_table.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "param or count_min or top_values or config4" > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
for P in slot rule; do
  SENTINEL_PARAM_PATH=$P timeout -k 10 240 python -u bench.py --config 4 --steps 20 --warmup 3 > $O/bench_4_$P.json 2> $O/bench_4_$P.err || { tail -20 $O/bench_4_$P.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_4_$P.json'));print('4 $P', d['value'], d['ms_per_step'], d['p99_batch_ms'], d.get('param_table'), {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
timeout -k 10 240 python -u bench.py --config 4cm --steps 20 --warmup 3 > $O/bench_4cm.json 2> $O/bench_4cm.err || { tail -20 $O/bench_4cm.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_4cm.json'));print('4cm', d['value'], d['ms_per_step'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()}, d.get('count_min'))"
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/b_c3.json 2> $O/b_c3.err || { tail -20 $O/b_c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/b_c3.json'));print('c3', round(d['value']/1e9,3), d['ms_per_step'], d['p99_batch_ms'], d['median_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
echo R02D OK
