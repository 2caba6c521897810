# GPU parity tests only (optionally a subset: bash scripts/gpu_tests_only.sh TAG tests/a.py tests/b.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-tests}
shift
mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest ${@:-tests} -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$TAG/tests.log 2>&1
rc=$?
tail -30 gpurun_out/$TAG/tests.log
exit $rc
