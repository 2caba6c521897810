# Param path after the slot-metadata change: parity (every param / reload / table test), config 4 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-param2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_param_rules_gpu.py tests/test_param_table.py tests/test_reload.py tests/test_gpu_parity.py tests/test_wire.py tests/test_cluster_abi.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 240 python -u bench.py --config 4 --steps 20 --warmup 3 > $O/bench_4.json 2> $O/bench_4.err || { tail -20 $O/bench_4.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_4.json'));print('4', d['value'], d['ms_per_step'], d['p99_batch_ms'], d.get('param_table'), {k:v['avg_us'] for k,v in d['kernels'].items()})"
echo PARAM2 OK
