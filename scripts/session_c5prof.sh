set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o bench -- python3 bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/prof_c5.log 2>&1; rc=$?; echo "prof c5 rc=$rc"; cat $OUT/prof_c5/bench_kernel_stats.csv; exit $rc
