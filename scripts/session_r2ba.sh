#!/bin/bash
# toff pair as one dword-aligned 8-B load (default) vs two 4-B loads (MR_TOFF_SPLIT); parity on the default build, C4/C3 A/B
set -o pipefail
OUT=gpurun_out/r2ba; mkdir -p $OUT
export TMPDIR=/tmp
K="" FILES="tests/test_gpu_parity.py tests/test_gpu_large.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" split; do MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/c4_$v.json 2>&1; rc=$?; echo "c4 [$v] $(tail -1 $OUT/c4_$v.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
for rep in 1 2; do for v in "" split; do MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/c3_$v.json 2>&1; rc=$?; echo "c3 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c3_$v.json)"; [ $rc -eq 0 ] || exit $rc; done; done
