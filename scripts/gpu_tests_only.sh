set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/param1
timeout -k 10 400 python -u -m pytest tests/test_param_rules_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/param1/tests.log 2>&1
rc=$?
tail -25 gpurun_out/param1/tests.log
exit $rc
