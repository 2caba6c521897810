set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; echo "TESTS EXIT $?"
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "BENCH EXIT $?"
cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err; echo "PROF EXIT $?"
find $R/gpurun_out/prof -name "*stats*" | head
