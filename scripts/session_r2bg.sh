#!/bin/bash
# tile-aware song shards: full GPU suite, smoke, then the C4 per-rank layout probe with tiled shards
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
OUT=gpurun_out/r2bg; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u scripts/layout_probe.py ibm 1x1,4x2,2x4 > $OUT/layouts_ibm_tiled.jsonl 2> $OUT/layouts_ibm_tiled.err; rc=$?
python -c "
import json
for l in open('$OUT/layouts_ibm_tiled.jsonl'):
    d=json.loads(l); print(d['layout'], round(d['max_rank_ms'],2), round(d['mean_rank_ms'],2), d['speedup_vs_1x1'] and round(d['speedup_vs_1x1'],2), [(x['n_tiles'], round(x['device_ms'],1)) for x in d['ranks']])
"; exit $rc
