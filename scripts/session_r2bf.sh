#!/bin/bash
# per-rank device time of the C4 multi-GPU layouts (one rank at a time on one GPU)
set -o pipefail
OUT=gpurun_out/r2bf; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 800 python -u scripts/layout_probe.py ibm 1x1,8x1,4x2,2x4,1x8 > $OUT/layouts_ibm.jsonl 2> $OUT/layouts_ibm.err; rc=$?
python -c "
import json
for l in open('$OUT/layouts_ibm.jsonl'):
    d=json.loads(l); print(d['layout'], round(d['max_rank_ms'],2), round(d['mean_rank_ms'],2), d['speedup_vs_1x1'] and round(d['speedup_vs_1x1'],2), [x['n_tiles'] for x in d['ranks']], round(d['wall_s'],1))
"; exit $rc
