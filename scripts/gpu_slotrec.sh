# Param slot records (SlotRec): full GPU parity (records on), then config 4 with records on / off and
# configs 3 and 2 (KeyTable gained a field: no change expected on the flow paths).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02_slotrec}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
run() {  # name config env...
  local name=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$name.json'));print('$name', round(d['value']/1e9,3), d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
}
run 4_rec 4 SENTINEL_SLOT_REC=1
run 4_norec 4 SENTINEL_SLOT_REC=0
run 3 3
run 2 2
echo SLOTREC OK
