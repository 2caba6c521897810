# Parity tests of the param table / config 2 at full size, then the drop-in path and every BASELINE
# config's bench line.  Usage (from gpurun): bash scripts/gpu_configs.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-configs}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_param_table.py tests/test_batcher.py tests/test_gpu_parity.py::test_config2_full_size_bitexact -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -12 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for M in sync async; do
  timeout -k 10 60 ./tools/dropin_bench --threads 32 --seconds 5 --mode $M --inflight 64 > $O/dropin_$M.json 2> $O/dropin_$M.err || { tail -5 $O/dropin_$M.err; exit 1; }
  cat $O/dropin_$M.json
done
for C in 2 5 3lim 4 4cm; do
  timeout -k 10 240 python -u bench.py --config $C --steps 20 --warmup 3 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C', d['value'], d['p99_batch_ms'], d['p99_sync_ms'], d['roofline'] and d['roofline']['kernel'], d['roofline'] and d['roofline']['frac'], d.get('count_min'), d['cpu_baseline'] and d['cpu_baseline']['value'])"
done
echo CONFIGS OK
