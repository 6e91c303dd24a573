#!/bin/bash
# wide kernel epilogue: scale loads of the next batch in flight (default) vs one batch at a time (base);
# parity of the wide / large sets on the default, then C3 / C4 / C5 A/B
set -o pipefail
OUT=gpurun_out/r2be; mkdir -p $OUT
export TMPDIR=/tmp
K="wide or large or chunk or ensemble" FILES="tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_gpu_ensemble.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" base; do MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/c3_$v.json 2>&1; rc=$?; echo "c3 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c3_$v.json)"; [ $rc -eq 0 ] || exit $rc; done; done
for rep in 1 2; do for v in "" base; do MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/c4_$v.json 2>&1; rc=$?; echo "c4 [$v] $(tail -1 $OUT/c4_$v.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
for v in "" base; do MR_ENGINE_LIB=$v timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c5_$v.json 2>&1; rc=$?; echo "c5 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_$v.json)"; [ $rc -eq 0 ] || exit $rc; done
