# Parity (flow paths, reload), then configs 2 / 5 / 3 bench lines.  Usage: bash scripts/gpu_het2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-het2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_reload.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
for C in 2 5 3; do
  timeout -k 10 240 python -u bench.py --config $C --steps 10 --warmup 2 --no-host-path --no-cpu-baseline --latency-batches 20 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C', d['value'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
echo HET2 OK
