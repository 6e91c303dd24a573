set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r2_c2 -o bench -- python3 bench.py --no-cpu-baseline --no-e2e > $OUT/prof_r2_c2.log 2>&1; rc=$?; echo "prof c2 rc=$rc"; cat $OUT/prof_r2_c2/bench_kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_r2_c2_$tag -o p -- python3 bench.py --no-cpu-baseline --no-e2e --steps 50 --warmup 5 > $OUT/pmc_r2_c2_$tag.log 2>&1; rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_traffic.py c2 "k_score<1, float, true>" $OUT/pmc_r2_c2.json $OUT/pmc_r2_c2_* | head -30
timeout -k 10 300 python bench.py > $OUT/r2i_bench_c2.json 2> $OUT/r2i_bench_c2.err; rc=$?; echo "bench rc=$rc"; cut -c1-300 $OUT/r2i_bench_c2.json; exit $rc
