set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SEL=${SEL:-}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread $SEL > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit $rc
