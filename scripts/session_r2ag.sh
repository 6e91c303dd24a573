#!/bin/bash
# C4 stage-1 chunk sweep (train users per k_neighbours LDS chunk), ibm and ubm, one 704-user batch
set -o pipefail
OUT=gpurun_out/r2ag; mkdir -p $OUT
export TMPDIR=/tmp
for model in ibm ubm; do for rep in 1 2; do for ch in 8192 4096 16384 2048; do MR_PROBE_CHUNK=$ch timeout -k 10 300 python scripts/c4_probe.py 704 $model > $OUT/c4_$ch.json 2>&1; rc=$?; echo "c4 $model chunk=$ch $(tail -1 $OUT/c4_$ch.json | grep -o '"device_ms": [0-9.]*\|"n_chunks": [0-9]*\|"batch": [0-9]*' | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done; done; done
