# A/B of an engine environment switch on one box: parity tests with the switch on, then the bench at
# the 1M-flow and 125k-flow (N=8 per-rank) shapes, off/on alternated twice.
# Usage (from gpurun): bash scripts/gpu_ab_env.sh TAG VAR VALUE
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=$1; VAR=$2; VAL=$3
O=gpurun_out/$TAG
mkdir -p $O
env $VAR=$VAL timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_reload.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/tests.log | head; exit $rc; }
for rep in 1 2; do
  for v in 0 $VAL; do
    for F in 1000000 125000; do
      env $VAR=$v timeout -k 10 120 python -u bench.py --flows $F --steps 20 --warmup 3 --no-cpu-baseline --no-host-path --latency-batches 50 > $O/b_${v}_${F}_$rep.json 2> $O/b_${v}_${F}_$rep.err || { tail -5 $O/b_${v}_${F}_$rep.err; exit 1; }
      python -c "import json;d=json.load(open('$O/b_${v}_${F}_$rep.json'));print('$VAR=$v F=$F', round(d['value']/1e9,2), {k:v['avg_us'] for k,v in d['kernels'].items()})"
    done
  done
done
# per-workgroup phase stamps of k_part_half (diagnostic build) at both shapes, switch off / on
for F in 1000000 125000; do
  for v in 0 $VAL; do
    env $VAR=$v SENTINEL_LIB=$GRAFT_REPO_ROOT/sentinel_amd/libsentinel_diag.so DIAG_FLOWS=$F timeout -k 10 120 python -u scripts/diag_phases.py > $O/phases_${v}_$F.txt 2>&1 || { tail -5 $O/phases_${v}_$F.txt; exit 1; }
    echo "$VAR=$v F=$F"; cat $O/phases_${v}_$F.txt | grep -v amdgpu.ids
  done
done
echo AB OK
