set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/r2m_bench_c2.json 2> $OUT/r2m_bench_c2.err; rc=$?; echo "bench c2 rc=$rc"; cut -c1-200 $OUT/r2m_bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/r2m_bench_c3.json 2> $OUT/r2m_bench_c3.err; rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c4 --steps 3 --warmup 1 > $OUT/r2m_bench_c4.json 2> $OUT/r2m_bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r2m_bench_c5.json 2> $OUT/r2m_bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; exit $rc
