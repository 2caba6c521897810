# Config 2 (and 5) on both flow paths.  Usage (from gpurun): bash scripts/gpu_cfg2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-cfg2}
O=gpurun_out/$TAG
mkdir -p $O
for C in 2 5; do
  for P in sorted partition; do
    SENTINEL_FLOW_PATH=$P timeout -k 10 240 python -u bench.py --config $C --steps 10 --warmup 2 --no-host-path --no-cpu-baseline --latency-batches 20 > $O/bench_${C}_$P.json 2> $O/bench_${C}_$P.err || { tail -20 $O/bench_${C}_$P.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench_${C}_$P.json'));print('$C $P', d['value'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done
echo CFG2 OK
