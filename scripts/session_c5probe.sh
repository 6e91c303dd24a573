set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python scripts/c5_probe.py > $OUT/c5_probe.log 2>&1; rc=$?; echo "probe rc=$rc"; tail -45 $OUT/c5_probe.log; exit $rc
