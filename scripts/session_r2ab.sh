#!/bin/bash
# refresh of the bulk lines after the 8-B segment loads: C3 / C4 / C5 bench + rocprof summaries
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2ab; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/bench_c3.json 2> $OUT/bench_c3.err; rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o bench -- python3 bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > $OUT/prof_c3.log 2>&1; rc=$?; echo "prof c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c4 --steps 3 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o bench -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_c4.log 2>&1; rc=$?; echo "prof c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o bench -- python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_c5.log 2>&1; rc=$?; echo "prof c5 rc=$rc"; exit $rc
