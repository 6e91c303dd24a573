set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_api_mirror.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/r2a_api.log 2>&1; rc=$?; echo "api rc=$rc"; tail -5 $OUT/r2a_api.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_large.py -m gpu -x -v --durations=0 --timeout 600 --timeout-method thread > $OUT/r2a_large.log 2>&1; rc=$?; echo "large rc=$rc"; tail -25 $OUT/r2a_large.log; exit $rc
