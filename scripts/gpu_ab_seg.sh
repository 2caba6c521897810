# Segment-kernel variants (SENTINEL_SEG_IMPL 0 LDS-staged / 1 256x16 vector runs / 2 512x8) and byte
# routes (SENTINEL_ROUTE8) on the radix-path configs: full GPU parity first (defaults), then A/B lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02_seg}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
run() {  # name config env...
  local name=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$name.json'));print('$name', round(d['value']/1e9,3), d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
}
for C in 3lim 2 5 4; do
  for S in 0 1 2; do run ${C}_s$S $C SENTINEL_SEG_IMPL=$S; done
done
run 3lim_r0 3lim SENTINEL_ROUTE8=0
echo AB OK
