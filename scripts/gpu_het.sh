# Parity (flow paths, reload) then the bench at the 1M / 125k config-3 shapes and config 5 (with a
# kernel trace of config 5).  Usage (from gpurun): bash scripts/gpu_het.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-het}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_reload.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
for F in 1000000 125000; do
  timeout -k 10 120 python -u bench.py --flows $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --latency-batches 50 > $O/b_$F.json 2> $O/b_$F.err || { tail -5 $O/b_$F.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$F.json'));print('F=$F', round(d['value']/1e9,2), {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 2 --no-host-path --latency-batches 50 > $O/bench_5.json 2> $O/bench_5.err || { tail -20 $O/bench_5.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_5.json'));print('5', d['value'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()}, d['cpu_baseline'] and d['cpu_baseline']['value'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof5 -o run -- python -u bench.py --config 5 --steps 5 --warmup 1 --no-host-path --no-cpu-baseline --latency-batches 5 --no-profile > $O/prof5.log 2>&1 || { tail -20 $O/prof5.log; exit 1; }
f=$(find $O/prof5 -name "*kernel_stats.csv" | head -1); python -c "
import csv,sys
r=list(csv.DictReader(open('$f')))
r.sort(key=lambda x:-float(x['TotalDurationNs']))
for x in r[:14]: print(x['Name'][:60], x['Calls'], round(float(x['AverageNs'])/1000,1))"
for H in 512 16384; do
  SENTINEL_HOT_HET_RUN=$H timeout -k 10 240 python -u bench.py --config 5 --steps 10 --warmup 2 --no-host-path --no-cpu-baseline --latency-batches 20 > $O/bench_5_$H.json 2> $O/bench_5_$H.err || { tail -20 $O/bench_5_$H.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_5_$H.json'));print('5 hot=$H', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
echo HET OK
