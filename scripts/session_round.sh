set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/session_refresh.sh; rc=$?; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o bench -- python3 bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $OUT/prof_c3.log 2>&1; rc=$?; echo "prof c3 rc=$rc"; cat $OUT/prof_c3/bench_kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o bench -- python3 bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof_c4.log 2>&1; rc=$?; echo "prof c4 rc=$rc"; cat $OUT/prof_c4/bench_kernel_stats.csv; exit $rc
