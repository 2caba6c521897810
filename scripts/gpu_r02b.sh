# Param fixes + staged verdicts: parity first, then A/B benches (SENTINEL_VSTAGE=0/1) and config 4.
# Usage (from gpurun): bash scripts/gpu_r02b.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02b}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 python -u scripts/debug_cm.py > $O/debug_cm.log 2>&1; tail -16 $O/debug_cm.log
timeout -k 10 400 python -u -m pytest tests/test_param_rules_gpu.py tests/test_param_table.py tests/test_gpu_parity.py tests/test_flow_batches.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -4 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
for F in 1000000 125000; do
  for V in 1 0; do
    SENTINEL_VSTAGE=$V timeout -k 10 200 python -u bench.py --flows $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/b_${F}_v$V.json 2> $O/b_${F}_v$V.err || { tail -20 $O/b_${F}_v$V.err; exit 1; }
    python -c "import json;d=json.load(open('$O/b_${F}_v$V.json'));print('$F v$V', round(d['value']/1e9,3), d['ms_per_step'], d['roofline']['avg_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
  done
done
for name in sg pg0; do
  SENTINEL_LIB=$GRAFT_REPO_ROOT/_variants/lib_$name.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/b_$name.json 2> $O/b_$name.err || { tail -20 $O/b_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$name.json'));print('$name', round(d['value']/1e9,3), d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
for C in 4 4cm; do
  timeout -k 10 240 python -u bench.py --config $C --steps 20 --warmup 3 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));print('$C', d['value'], d['ms_per_step'], d['p99_batch_ms'], d.get('param_table'), {k:v['avg_us'] for k,v in d['kernels'].items()}, d.get('count_min'))"
done
echo R02B OK
