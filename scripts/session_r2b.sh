set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_group.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/r2b_group.log 2>&1; rc=$?; echo "group rc=$rc"; tail -25 $OUT/r2b_group.log; exit $rc
