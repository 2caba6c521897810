# Quick bench + rocprofv3 kernel trace of a short bench run; prints per-kernel durations and the
# idle gaps between consecutive kernels of the last steps (launch / event overheads).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/gaps
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-host-path > gpurun_out/gaps/bench.json 2> gpurun_out/gaps/bench.err || { tail -5 gpurun_out/gaps/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/gaps/bench.json'));print(d['value'], d['ms_per_step'], d['p99_batch_ms'], {k:v['avg_us'] for k,v in d['kernels'].items()})"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/gaps/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > /dev/null 2> $R/gpurun_out/gaps/prof.err || { tail -5 $R/gpurun_out/gaps/prof.err; exit 1; }
cd $R
python scripts/trace_gaps.py gpurun_out/gaps/prof/run_kernel_trace.csv
