#!/bin/bash
# C5 bench line on the final tree (10 timed steps, two-hop CPU baseline on the usable cores)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2bp; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 700 python bench.py --config c5 --steps 10 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; grep -o '"ms_per_step": [0-9.]*\|"frac": [0-9.]*' $OUT/bench_c5.json; exit $rc
