#!/bin/bash
# wide kernel retune after the 8-B segment loads: kSeg 8/12/16, R 1/2/3 (C4 batch + C3 step)
set -o pipefail
OUT=gpurun_out/r2y; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do for v in "" seg8 seg16 r3 r1; do MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/c4_$v.json 2>&1; rc=$?; echo "c4 [$v] $(tail -1 $OUT/c4_$v.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
for v in "" seg8 seg16 r3 r1; do MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/c3_$v.json 2>&1; rc=$?; echo "c3 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c3_$v.json)"; [ $rc -eq 0 ] || exit $rc; done
