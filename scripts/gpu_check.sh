# GPU round check: parity tests, then bench, then a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
echo "== tests"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 \
  && tail -3 gpurun_out/gpu_tests.log \
  && echo "== bench" \
  && timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err \
  && cat gpurun_out/bench.json \
  && echo "== rocprof" \
  && cd /tmp && export TMPDIR=/tmp \
  && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/bench_prof.json 2> $R/gpurun_out/prof.err \
  && echo "PROF OK"
rc=$?
echo "EXIT $rc"
tail -30 $R/gpurun_out/gpu_tests.log | grep -E "Error|assert|FAIL|passed|failed" | head -10
exit $rc
