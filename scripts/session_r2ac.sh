#!/bin/bash
# C4 / C3 per-step HBM traffic for the bench lines: FETCH_SIZE, WRITE_SIZE, TCC hit/miss passes over bench steps
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2ac; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in c3 c4; do
  if [ $cfg = c4 ]; then B="bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e"; N=1; else B="bench.py --config c3 --steps 3 --warmup 0 --no-cpu-baseline --no-e2e"; N=3; fi
  for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $pass | cut -d' ' -f1)
    timeout -s KILL 400 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_${cfg}_$tag -o p -- python3 $B > $OUT/pmc_${cfg}_$tag.log 2>&1; rc=$?; echo "pmc $cfg $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python scripts/pmc_traffic.py $cfg step:$N $OUT/pmc_$cfg.json $OUT/pmc_${cfg}_* > /dev/null || exit 1
  grep -E '"traffic_bytes_per_launch"|"l2_hit_rate"|"dispatches"' -A0 $OUT/pmc_$cfg.json
done
