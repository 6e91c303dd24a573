#!/bin/bash
# C5 per-step PMC traffic, then the C3 / C4 / C5 bench lines carrying the measured traffic
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2ad; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B="bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 400 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_c5_$tag -o p -- python3 $B > $OUT/pmc_c5_$tag.log 2>&1; rc=$?; echo "pmc c5 $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_traffic.py c5 step:1:k_topk_dense $OUT/pmc_c5.json $OUT/pmc_c5_* > /dev/null || exit 1
cp $OUT/pmc_c5.json profiles/pmc_c5.json
grep -E '"traffic_bytes_per_launch"|"l2_hit_rate"' $OUT/pmc_c5.json
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_c3.json 2> $OUT/bench_c3.err; rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; exit $rc
