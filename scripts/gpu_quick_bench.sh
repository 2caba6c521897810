# GPU parity tests (optional subset) + a quick bench per flow-path variant (no profiler).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-quick}
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/tests.log; grep -E "^E |Error|FAILED" gpurun_out/$TAG/tests.log | head -12
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-partition sorted}; do
  SENTINEL_FLOW_PATH=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench_$v.json 2>gpurun_out/$TAG/bench_$v.err || { tail -5 gpurun_out/$TAG/bench_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/$TAG/bench_$v.json'));print('$v', d['value'], d['p99_batch_ms'], d['roofline']['kernel'], d['roofline']['frac'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
