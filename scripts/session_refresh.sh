set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="bench.py --no-cpu-baseline --config c2 --steps 50 --warmup 5"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_c2_$tag -o p -- python3 $B > $OUT/pmc_c2_$tag.log 2>&1; rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py "k_score<1, float, true>" $OUT/pmc_c2_* > $OUT/pmc_c2_summary.json; cat $OUT/pmc_c2_summary.json
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err; rc=$?; echo "bench c2 rc=$rc"; cat $OUT/bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o bench -- python3 bench.py --no-cpu-baseline --steps 200 > $OUT/prof_c2.log 2>&1; rc=$?; echo "prof c2 rc=$rc"; cat $OUT/prof_c2/bench_kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_c3.json 2>/dev/null; rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python bench.py --config c5 --steps 2 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; exit $rc
