# PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes) of the other BASELINE configs' shapes, then
# their bench lines again so `roofline.traffic` is measured on each config's own shape.
# usage (from gpurun): bash scripts/gpu_pmc_configs.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r02_cfg}
O=gpurun_out/$TAG
mkdir -p $O
for C in ${PMC_CONFIGS:-2 5 3lim 4}; do
  bash scripts/gpu_pmc_shape.sh ${TAG}_c$C --config $C > $O/pmc_$C.log 2>&1 || { tail -20 $O/pmc_$C.log; exit 1; }
done
for C in 2 5 3lim 4; do
  timeout -k 10 240 python -u bench.py --config $C --steps 20 --warmup 3 > $O/bench_$C.json 2> $O/bench_$C.err || { tail -20 $O/bench_$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$C.json'));r=d['roofline'];print('$C', round(d['value']/1e9,3), d['p99_batch_ms'], r['kernel'], r['frac'], r['traffic'], r['algorithmic_bytes_per_launch'])"
done
echo PMCCFG OK
