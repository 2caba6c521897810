# Cost diagnostics: linear (wrong-order) verdict writes, and FETCH/WRITE counters per kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
SENTINEL_DIAG_LINEAR=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/diag_linear.json 2>gpurun_out/diag_linear.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/diag_linear.json'));print('linear', d['value'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > /dev/null 2>$R/gpurun_out/pmc_fetch.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > /dev/null 2>$R/gpurun_out/pmc_write.err || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $R/gpurun_out/pmc_hit -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile > /dev/null 2>$R/gpurun_out/pmc_hit.err || exit 1
echo PMC OK
