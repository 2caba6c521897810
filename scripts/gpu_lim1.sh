# Limiter prep A/B: the limiter / namespace parity tests, then config 3lim with the fused one-limiter
# prep (default) and with prep + radix pass (SENTINEL_LIM1=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02_lim1}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "limiter or namespace or invalid" --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
for L in 1 0; do
  SENTINEL_LIM1=$L timeout -k 10 300 python -u bench.py --config 3lim --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_3lim_l$L.json 2> $O/bench_3lim_l$L.err || { tail -20 $O/bench_3lim_l$L.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_3lim_l$L.json'));print('l$L', round(d['value']/1e9,3), d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
echo LIM1 OK
