# Round-6 A/B call: flow parity (every pipeline incl. decide-order from the partition and radix paths),
# configs 2 / 5 in decide order vs arrival order, and the count-min block walk's sub-range bits.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_ab
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_batcher.py -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
for c in 2 5; do for o in arrival decide; do
  timeout -k 10 200 python -u bench.py --config $c --output $o --no-cpu-baseline --no-host-path > $O/bench_${c}_$o.json 2> $O/bench_${c}_$o.err || { tail -20 $O/bench_${c}_$o.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_${c}_$o.json')); print('$c $o', d['value'], d['ms_per_step'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done; done
for sb in 0 2 3; do
  SENTINEL_CM_SB=$sb timeout -k 10 300 python -u bench.py --config 4cm --no-cpu-baseline --no-host-path > $O/bench_4cm_sb$sb.json 2> $O/bench_4cm_sb$sb.err || { tail -20 $O/bench_4cm_sb$sb.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_4cm_sb$sb.json')); print('4cm sb$sb', d['value'], d['ms_per_step'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()}, d['count_min']['violations'])"
done
echo DONE
