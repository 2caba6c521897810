# Parity of the flow paths, then the bench at the per-rank shapes (1M, 500k, 250k, 125k flows) and
# the k_part_half phase stamps.  Usage (from gpurun): bash scripts/gpu_shapes.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-shapes}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
for F in 1000000 500000 250000 125000; do
  timeout -k 10 120 python -u bench.py --flows $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --latency-batches 50 > $O/b_$F.json 2> $O/b_$F.err || { tail -5 $O/b_$F.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$F.json'));print('F=$F', round(d['value']/1e9,2), {k:v['avg_us'] for k,v in d['kernels'].items()})"
done
for F in 1000000 125000; do
  SENTINEL_LIB=$GRAFT_REPO_ROOT/sentinel_amd/libsentinel_diag.so DIAG_FLOWS=$F timeout -k 10 120 python -u scripts/diag_phases.py > $O/phases_$F.txt 2>&1 || { tail -5 $O/phases_$F.txt; exit 1; }
  echo "F=$F"; grep -v amdgpu.ids $O/phases_$F.txt | grep -v "times:"
done
echo SHAPES OK
