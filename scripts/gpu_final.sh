# Round evidence: every GPU test, the config-3 bench + rocprof + PMC of its shape (gpu_round.sh), then
# the other BASELINE configs' bench lines.  Usage (from gpurun): bash scripts/gpu_final.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-final}
bash scripts/gpu_round.sh $TAG ${2:-} || exit $?
O=gpurun_out/$TAG
for C in 2 5 3lim 4 4cm; do
  timeout -k 10 240 python -u bench.py --config $C --steps 20 --warmup 3 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C', d['value'], d['p99_batch_ms'], d['roofline'] and d['roofline']['kernel'], d['roofline'] and d['roofline']['frac'], d.get('count_min', {}) and d['count_min'].get('violations'))"
done
echo FINAL OK
