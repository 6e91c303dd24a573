#!/bin/bash
# stage 1 over G chunks per workgroup (k_neighbours_multi, default G=4) vs one chunk per workgroup (g1), G=2/8;
# parity (chunked stage 1, wide, large) on the default, then the C4 one-batch A/B
set -o pipefail
OUT=gpurun_out/r2bh; mkdir -p $OUT
export TMPDIR=/tmp
K="wide or large or chunk or neighbour or group" FILES="tests/test_gpu_parity.py tests/test_gpu_large.py tests/test_group.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" g1 g2 g8; do MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/c4_$v.json 2>&1; rc=$?; echo "c4 [$v] $(tail -1 $OUT/c4_$v.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
for v in "" g1; do MR_ENGINE_LIB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$v -o p -- python3 scripts/c4_probe.py 704 > $OUT/prof_$v.log 2>&1; rc=$?; echo "prof [$v] rc=$rc"; grep -h "k_neighbours" $OUT/prof_$v/p_kernel_stats.csv | cut -c1-160; [ $rc -eq 0 ] || exit $rc; done
