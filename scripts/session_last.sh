set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err; rc=$?; echo "bench c2 rc=$rc"; cut -c1-400 $OUT/bench_c2.json; exit $rc
