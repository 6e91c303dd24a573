#!/bin/bash
# C3 / C4 bench lines after the baseline fixes (two-hop CPU baseline at C3, vs_baseline only at C2)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r2final; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err; rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 10 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
for c in ("c3", "c4"):
    d = json.loads(open(f"gpurun_out/r2final/bench_{c}.json").read().strip().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    print(c, "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "frac %.4f" % d["roofline"]["frac"], "vs", d["vs_baseline"], "cpu", cb.get("value"), cb.get("cores"))
PY
