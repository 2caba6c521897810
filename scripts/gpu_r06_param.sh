# Round-6: decide-order output of the param key walks -- param suites (exact with both outputs, count-min,
# wire server) and configs 4 / 4cm in arrival vs decide order.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_param
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_param_table.py tests/test_param_rules_gpu.py tests/test_wire.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
for c in 4 4cm; do for o in arrival decide; do
  timeout -k 10 300 python -u bench.py --config $c --output $o --no-cpu-baseline --no-host-path > $O/bench_${c}_$o.json 2> $O/bench_${c}_$o.err || { tail -20 $O/bench_${c}_$o.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_${c}_$o.json')); print('$c $o', d['value'], d['ms_per_step'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()}, d.get('count_min', {}).get('violations'))"
done; done
echo DONE
