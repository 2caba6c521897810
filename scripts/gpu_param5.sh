# Param header loads issued with the key's n (bucketed slot stride): full GPU parity, then configs 4,
# 2 and 5 (the radix-path flow tables take the same k_process_reg change).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02_param5}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
for C in 4 2 5; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C', round(d['value']/1e9,3), d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
echo PARAM5 OK
