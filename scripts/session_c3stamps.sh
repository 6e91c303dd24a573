set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
CONFIG=c3 DENSE=1 timeout -k 10 300 python scripts/large_stamps.py 0 0 ibm > $OUT/c3_stamps.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/c3_stamps.log | head -40; exit $rc
