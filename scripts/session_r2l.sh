set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MR_ENGINE_LIB=pipe K="wide" FILES="tests/test_gpu_parity.py" bash scripts/session_tests.sh || exit $?
timeout -k 10 400 python scripts/c4_probe.py 704 > $OUT/r2l_warm.json 2>&1; rc=$?; tail -1 $OUT/r2l_warm.json | cut -c1-150; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in "" pipe pipe_r2 pref; do MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/r2l_$v.json 2>&1; rc=$?; echo "[$v] $(tail -1 $OUT/r2l_$v.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
