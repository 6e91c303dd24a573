set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 300 --timeout-method thread -k "chunks or wide or large_train or c3_scale" > gpurun_out/pytest_large.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_large.log
[ $rc -eq 0 ] || exit $rc
for a in "$@"; do
  timeout -k 10 400 python scripts/large_probe.py $a > gpurun_out/probe.log 2>&1; rc=$?; grep -E "dataset|load|run 2|exact" gpurun_out/probe.log; [ $rc -eq 0 ] || exit $rc
done
