set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06_c3
mkdir -p $O
cd $R
echo "== bench (decide order, full)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "== rocprof stats"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-path > $O/bench_prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
cd $R
python scripts/trace_summary.py $O/prof/run_kernel_trace.csv warmup:2,profile:3,timed:10 > $O/kernel_trace_summary.json
echo "== pmc"
bash scripts/gpu_pmc_req.sh r06_c3 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-host-path > $O/pmc_req.log 2>&1 || { tail -20 $O/pmc_req.log; exit 1; }
rm -rf $R/gpurun_out/pmcreq_r06_c3/rd $R/gpurun_out/pmcreq_r06_c3/wr
echo "== configs 2 / 5: auto vs forced partition"
for c in 2 5; do
  timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-host-path > $O/bench_$c.json 2> $O/bench_$c.err || { tail -20 $O/bench_$c.err; exit 1; }
  SENTINEL_FLOW_PATH=partition timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --no-host-path > $O/bench_${c}_part.json 2> $O/bench_${c}_part.err || { tail -20 $O/bench_${c}_part.err; exit 1; }
done
echo DONE
