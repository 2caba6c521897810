# Parity (partition + stream cases) on the in-tree build, then A/B bench of _variants/lib_*.so
# (LIBS="name ..."), then the phase stamps of the *_ph variants (PH="name ...").
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/ab
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/ab/tests.log 2>&1
rc=$?; tail -2 gpurun_out/ab/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/ab/tests.log | head; exit $rc; }
for name in ${LIBS}; do
  SENTINEL_LIB=$R/_variants/lib_$name.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path ${BENCH_ARGS} > gpurun_out/ab/$name${BTAG}.json 2>gpurun_out/ab/$name.err || { tail -5 gpurun_out/ab/$name.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ab/$name${BTAG}.json'));print('$name', round(d['value']/1e9,3), d['roofline']['avg_us'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
for name in ${PH}; do
  SENTINEL_LIB=$R/_variants/lib_$name.so timeout -k 10 200 python -u scripts/diag_phases.py > gpurun_out/ab/ph_$name.log 2>&1 || { tail -5 gpurun_out/ab/ph_$name.log; exit 1; }
  echo "== $name"; cat gpurun_out/ab/ph_$name.log | grep -v amdgpu.ids
done
