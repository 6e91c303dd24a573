#!/bin/bash
# HIP-graph replay: parity tests, then C2 / C1 bench with and without --graph (same box)
set -o pipefail
mkdir -p gpurun_out/r2u
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_graph.py > gpurun_out/r2u/test_graph.log 2>&1 || { tail -30 gpurun_out/r2u/test_graph.log; exit 1; }
tail -3 gpurun_out/r2u/test_graph.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --steps 2000 --no-graph > gpurun_out/r2u/c2_plain_$i.json || exit 1
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --steps 2000 --graph > gpurun_out/r2u/c2_graph_$i.json || exit 1
done
timeout -k 10 200 python -u bench.py --config c1 --model ubm --no-cpu-baseline --no-e2e --steps 2000 --no-graph > gpurun_out/r2u/c1_plain.json || exit 1
timeout -k 10 200 python -u bench.py --config c1 --model ubm --no-cpu-baseline --no-e2e --steps 2000 --graph > gpurun_out/r2u/c1_graph.json || exit 1
python - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/r2u/*.json")):
    d=json.load(open(f)); print(f, round(d["ms_per_step"]*1e3,2), "us/step", "%.3e"%d["value"], d["config"].get("launch"))
P
