# Limiter on the partition path: full GPU parity, then the limiter-on bench, config 3 (full bench line,
# with the rule-reload leg) and config 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02e}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
for C in 4cm 4 2; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C', round(d['value']/1e9,3), d['ms_per_step'], d['p99_batch_ms'], d.get('rule_reload_ms'), {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
echo R02E OK
