#!/bin/bash
# fused kernel tile top-k: keys read from the epilogue registers (default) vs from LDS
# (tlds); full GPU suite + smoke on the default, then C2 A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r2bm; mkdir -p $OUT
export TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do for v in "" tlds; do MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --steps 2000 --warmup 100 > $OUT/c2_$v.json 2>&1; rc=$?; echo "c2 [$v] $(grep -o '"ms_per_step": [0-9.]*\|"avg_launch_us": [0-9.]*' $OUT/c2_$v.json | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc; done; done
