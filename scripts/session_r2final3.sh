#!/bin/bash
# round-2 final refresh after the fused-kernel top-k changes: every -m gpu test, smoke, C2 PMC traffic passes
# (copied to profiles/pmc_c2.json so the bench line reads them), the default bench line, its rocprof summary, C1
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2final3; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log $OUT/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
B="bench.py --no-cpu-baseline --no-e2e --config c2 --steps 50 --warmup 5"
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_c2_$tag -o p -- python3 $B > $OUT/pmc_c2_$tag.log 2>&1; rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_traffic.py c2 "k_score<1, float, true>" $OUT/pmc_c2.json $OUT/pmc_c2_* || exit 1
cp $OUT/pmc_c2.json profiles/pmc_c2.json
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err; rc=$?; echo "bench c2 rc=$rc"; cut -c1-400 $OUT/bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o bench -- python3 bench.py --no-cpu-baseline --no-e2e > $OUT/prof_c2.log 2>&1; rc=$?; echo "prof c2 rc=$rc"; head -3 $OUT/prof_c2/bench_kernel_stats.csv | cut -c1-160; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c1 --model ubm > $OUT/bench_c1_ubm.json 2> $OUT/bench_c1.err; rc=$?; echo "bench c1 rc=$rc"; exit $rc
