#!/bin/bash
# wide-kernel block -> (user, tile) maps: parity under MR_WIDE_MAP=3 and 0, then C4 one-batch A/B
# (map 1 = default: all tiles of a user on one XCD; 0 = hardware order; 2 = tile-major ranges per XCD;
#  3 = XCD x owns tiles x, x+8, ... for all users in order), 20 tiles (auto) and 24 tiles (16128 songs)
set -o pipefail
OUT=gpurun_out/r2bc; mkdir -p $OUT
export TMPDIR=/tmp
for m in 3 0; do MR_WIDE_MAP=$m K="wide or large or chunk" FILES="tests/test_gpu_parity.py tests/test_gpu_large.py" bash scripts/session_tests.sh || exit $?; cp gpurun_out/pytest_gpu.log $OUT/pytest_map$m.log; done
for rep in 1 2; do for cfg in "1 0" "0 0" "2 0" "3 16128" "1 16128" "0 16128"; do set -- $cfg; MR_WIDE_MAP=$1 MR_PROBE_BS=$2 timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/c4_m$1_b$2.json 2>&1; rc=$?; echo "c4 map $1 bs $2: $(tail -1 $OUT/c4_m$1_b$2.json | grep -o '"n_tiles": [0-9]*\|"device_ms": [0-9.]*' | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done; done
