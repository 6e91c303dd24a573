#!/bin/bash
# C2 wall-clock variance: one K-step graph vs 25- and 50-step graphs vs stream launches, 4 runs each
set -o pipefail
OUT=gpurun_out/r2ai; mkdir -p $OUT
for rep in 1 2 3 4; do
  for mode in "--graph-steps 0" "--graph-steps 50" "--graph-steps 20" "--no-graph"; do
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e $mode > $OUT/c2.json || exit 1
    echo "[$mode] $(python -c "import json;d=json.loads(open('$OUT/c2.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step']*1e3,2), 'us/step; device', round(d['roofline']['avg_launch_us'],2), 'us; submit', round(d['config']['host_submit_ms'],3), 'ms')")"
  done
done
