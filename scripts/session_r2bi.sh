#!/bin/bash
# threshold mAP on the device: only the label classes' ids / counts / AP cross PCIe, minmax scratch stream-ordered
# (default) vs the whole-shard pos / AP arrays (evbase); ensemble GPU tests, then C5 A/B
set -o pipefail
OUT=gpurun_out/r2bi; mkdir -p $OUT
export TMPDIR=/tmp
K="" FILES="tests/test_gpu_ensemble.py tests/test_gpu_large.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" evbase; do MR_ENGINE_LIB=$v timeout -k 10 400 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c5_$v.json 2>&1; rc=$?; echo "c5 [$v] $(grep -o '"ms_per_step": [0-9.]*\|"lcm": [0-9.e-]*' $OUT/c5_$v.json | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done; done
