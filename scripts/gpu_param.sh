# Param path checks + config 4 benches (exact / shared count-min) after the slot-table and sketch changes.
# Usage (from gpurun): bash scripts/gpu_param.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-param}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_param_rules_gpu.py tests/test_param_table.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k "param or count_min or config4 or top_values" > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
for C in 4 4cm; do
  timeout -k 10 240 python -u bench.py --config $C --steps 20 --warmup 3 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C', d['value'], d['ms_per_step'], d['p99_batch_ms'], d.get('param_table'), {k:v['avg_us'] for k,v in d['kernels'].items()}, d.get('count_min'))"
done
echo PARAM OK
