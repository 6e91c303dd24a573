#!/bin/bash
# wide kernel tile width: the widest tile (1 workgroup per CU, LDS-bound) vs tiles of <= 80 KiB LDS
# (2 x 1024-thread workgroups per CU: one's epilogue / top-k overlaps the other's walk), C3 and C4
set -o pipefail
OUT=gpurun_out/r2bd; mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1 2; do for bs in 0 9472 8192; do timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --block-songs $bs > $OUT/c3_b$bs.json 2>&1; rc=$?; echo "c3 bs $bs: $(grep -o '"ms_per_step": [0-9.]*\|"n_tiles": [0-9]*' $OUT/c3_b$bs.json | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done; done
for bs in 0 9472; do MR_PROBE_BS=$bs timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/c4_b$bs.json 2>&1; rc=$?; echo "c4 bs $bs: $(tail -1 $OUT/c4_b$bs.json | grep -o '"n_tiles": [0-9]*\|"device_ms": [0-9.]*' | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done
