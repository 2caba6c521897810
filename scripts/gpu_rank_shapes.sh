# Per-rank shapes of the scaling bench on one MI355X: bit-exact parity at rank 0's shard for
# N = 1, 2, 8, then the bench at the per-rank flow counts of N = 2, 4, 8 (1M / N flows, 8M events).
# Usage (from gpurun): bash scripts/gpu_rank_shapes.sh [TAG]   -> results under gpurun_out/$TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-rank_shapes}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread -k bench_rank_shapes > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
for F in 500000 250000 125000; do
  timeout -k 10 180 python -u bench.py --flows $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_$F.json 2> $O/bench_$F.err || { tail -20 $O/bench_$F.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$F.json')); print($F, d['value'], d['p99_batch_ms'], d['kernels'])"
done
echo "SHAPES OK"
