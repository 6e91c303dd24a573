#!/bin/bash
# bulk refresh after the DPP + 4096-user stage-1 chunks: per-step PMC (C4, C5), C3/C4/C5 bench lines + rocprof
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2aj; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in c4 c5; do
  if [ $cfg = c4 ]; then B="bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e"; X=""; else B="bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline"; X=":k_topk_dense"; fi
  for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 400 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_${cfg}_$tag -o p -- python3 $B > $OUT/pmc_${cfg}_$tag.log 2>&1; rc=$?; echo "pmc $cfg $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python scripts/pmc_traffic.py $cfg step:1$X $OUT/pmc_$cfg.json $OUT/pmc_${cfg}_* > /dev/null || exit 1
  cp $OUT/pmc_$cfg.json profiles/pmc_$cfg.json
  grep -E '"traffic_bytes_per_launch"|"l2_hit_rate"' $OUT/pmc_$cfg.json
done
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_c3.json 2> $OUT/bench_c3.err; rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o bench -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/prof_c3.log 2>&1; rc=$?; echo "prof c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o bench -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_c4.log 2>&1; rc=$?; echo "prof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o bench -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_c5.log 2>&1; rc=$?; echo "prof c5 rc=$rc"; exit $rc
