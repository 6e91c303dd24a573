set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
# K: optional pytest -k expression; FILES: optional test paths (default: tests)
if [ -n "${K:-}" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest ${FILES:-tests} -m gpu -x -q -rf --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_gpu.log; exit $rc
