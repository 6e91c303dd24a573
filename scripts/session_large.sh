set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -rf --timeout 300 --timeout-method thread -k "chunks or wide or large_train or tile_sizes" > gpurun_out/pytest_large.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_large.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/large_probe.py 100000 1000 ibm > gpurun_out/probe_100k.log 2>&1; rc=$?; cat gpurun_out/probe_100k.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/large_probe.py 1009318 1000 ibm > gpurun_out/probe_1m.log 2>&1; rc=$?; cat gpurun_out/probe_1m.log; exit $rc
