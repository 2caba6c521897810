# Stream-path parity test + one bench line (no profiler).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stream or config2" > gpurun_out/stream_tests.log 2>&1
rc=$?; tail -3 gpurun_out/stream_tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/stream_tests.log | head; exit $rc; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/stream_bench.json 2> gpurun_out/stream_bench.err || { tail -20 gpurun_out/stream_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/stream_bench.json'));print(d['value'],d['p99_batch_ms'],json.dumps(d['host_path']))"
