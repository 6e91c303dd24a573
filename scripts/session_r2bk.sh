#!/bin/bash
# fused kernel: tile / merge top-k lists written by the ranking threads straight to their global slots (default)
# vs through LDS + barrier + copy loop (vialds); full GPU suite on the default, then C2 / C1 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r2bk; mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in "" vialds; do MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 2000 --warmup 100 > $OUT/c2_$v.json 2>&1; rc=$?; echo "c2 [$v] $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' $OUT/c2_$v.json | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done; done
for v in "" vialds; do MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --config c1 --model ubm --no-cpu-baseline --no-e2e --steps 2000 --warmup 100 > $OUT/c1_$v.json 2>&1; rc=$?; echo "c1 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1_$v.json)"; [ $rc -eq 0 ] || exit $rc; done
