#!/bin/bash
# C2 fused tile width after the merge change (candidates in registers while n_tiles x 10 <= 256)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2bq; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rep in 1 2; do for bs in 0 1024 1280; do timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 2000 --warmup 100 --block-songs $bs > $OUT/c2_b$bs.json 2>&1; rc=$?; echo "c2 bs $bs: $(grep -o '"ms_per_step": [0-9.]*\|"n_tiles": [0-9]*' $OUT/c2_b$bs.json | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done; done
