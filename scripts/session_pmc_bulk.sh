set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -q -rf --timeout 400 --timeout-method thread > $OUT/pytest_multirank.log 2>&1; rc=$?; echo "multirank rc=$rc"; tail -5 $OUT/pytest_multirank.log; [ $rc -eq 0 ] || exit $rc
P="scripts/large_probe.py 1009318 1000 ibm"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_c4_$tag -o p -- python3 $P > $OUT/pmc_c4_$tag.log 2>&1; rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py k_score_wide $OUT/pmc_c4_* > $OUT/pmc_c4_score_wide.json; cat $OUT/pmc_c4_score_wide.json
python scripts/pmc_summary.py k_neighbours $OUT/pmc_c4_* > $OUT/pmc_c4_neighbours.json; cat $OUT/pmc_c4_neighbours.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o bench -- python3 bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $OUT/prof_c5.log 2>&1; rc=$?; echo "prof c5 rc=$rc"; cat $OUT/prof_c5/bench_kernel_stats.csv; exit $rc
