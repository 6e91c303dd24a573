#!/bin/bash
# device mAP fold: ensemble + large GPU tests, then C5 bench twice
set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2ak; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
K="" FILES="tests/test_gpu_ensemble.py tests/test_gpu_large.py tests/test_driver.py tests/test_api_mirror.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do
timeout -k 10 500 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c5.json)"; [ $rc -eq 0 ] || exit $rc
done
