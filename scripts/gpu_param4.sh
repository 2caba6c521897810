# Param process kernel occupancy: the param parity suites, then config 4 with k_process_reg held to 4
# waves per SIMD (default) and without (SENTINEL_PROC_OCC=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02_param4}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_param_rules_gpu.py tests/test_param_table.py tests/test_gpu_parity.py -m gpu -x -v -k "param or Param" --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head -20; exit $rc; }
run() {  # name config env...
  local name=$1 c=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$name.json'));print('$name', round(d['value']/1e9,3), d['ms_per_step'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
}
run 4_occ 4
run 4_noocc 4 SENTINEL_PROC_OCC=0
echo PARAM4 OK
