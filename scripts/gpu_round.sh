# Full GPU round check on one MI355X: parity tests, bench, rocprofv3 kernel stats, and the PMC
# traffic of the bench's own shape (scripts/gpu_pmc_req.sh: the memory-side request counters by size in
# two separate passes, summarised into gpurun_out/pmcreq_<TAG>_c3/summary.json).
# Every GPU step has its own time limit; the chain stops at the first failure.
# Usage (from gpurun): bash scripts/gpu_round.sh [TAG] [--shapes]   -> results under gpurun_out/$TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-round}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
echo "== tests"
timeout -k 10 480 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/gpu_tests.log | head -20; exit $rc; }
echo "== bench"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
if [ "$2" = "--shapes" ]; then
  echo "== per-rank shapes of the scaling bench (1M / N flows per rank, 8M events)"
  for F in 500000 250000 125000; do
    timeout -k 10 180 python -u bench.py --flows $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_flows_$F.json 2> $O/bench_flows_$F.err || { tail -20 $O/bench_flows_$F.err; exit 1; }
  done
  python -c "import json; print(json.dumps({F: {k: json.load(open('$O/bench_flows_%d.json' % F))[k] for k in ('value', 'p99_batch_ms', 'kernels')} for F in (500000, 250000, 125000)}))" > $O/rank_shapes.json && cat $O/rank_shapes.json
fi
echo "== rocprof stats"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > $O/bench_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cd $R
python scripts/trace_summary.py $O/prof/run_kernel_trace.csv warmup:2,profile:3,timed:10 > $O/kernel_trace_summary.json
echo "== pmc (bench shape, memory-side requests by size)"
bash scripts/gpu_pmc_req.sh ${TAG}_c3 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-host-path > $O/pmc_req.log 2>&1 || { tail -20 $O/pmc_req.log; exit 1; }
rm -rf $R/gpurun_out/pmcreq_${TAG}_c3/rd $R/gpurun_out/pmcreq_${TAG}_c3/wr
echo "ROUND OK"
