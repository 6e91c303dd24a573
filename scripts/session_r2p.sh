set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r2_c3 -o bench -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/prof_r2_c3.log 2>&1; rc=$?; echo "prof c3 rc=$rc"; cat $OUT/prof_r2_c3/bench_kernel_stats.csv | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r2_c4 -o bench -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_r2_c4.log 2>&1; rc=$?; echo "prof c4 rc=$rc"; cat $OUT/prof_r2_c4/bench_kernel_stats.csv | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r2_c5 -o bench -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_r2_c5.log 2>&1; rc=$?; echo "prof c5 rc=$rc"; cat $OUT/prof_r2_c5/bench_kernel_stats.csv | cut -c1-160; exit $rc
