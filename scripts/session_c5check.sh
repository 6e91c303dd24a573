set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 600 python bench.py --config c5 --steps 3 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c5.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o bench -- python3 bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof_c5.log 2>&1; rc=$?; echo "prof c5 rc=$rc"; cat $OUT/prof_c5/bench_kernel_stats.csv; exit $rc
