#!/bin/bash
# round-2 refresh on the final tree: GPU suite, smoke, default C2 bench + rocprof, C3/C4/C5 bench lines
# (C4/C5 with >= 10 timed steps; the two-hop CPU baseline on all usable cores)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r2final; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log $OUT/
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err; rc=$?; echo "bench c2 rc=$rc"; cut -c1-300 $OUT/bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o bench -- python3 bench.py --no-cpu-baseline --no-e2e --steps 200 > $OUT/prof_c2.log 2>&1; rc=$?; echo "prof c2 rc=$rc"; cut -c1-150 $OUT/prof_c2/bench_kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c1 --model ubm > $OUT/bench_c1_ubm.json 2> $OUT/bench_c1.err; rc=$?; echo "bench c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err; rc=$?; echo "bench c3 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 10 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python bench.py --config c5 --steps 10 --warmup 3 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
for c in ("c1_ubm", "c2", "c3", "c4", "c5"):
    d = json.loads(open(f"gpurun_out/r2final/bench_{c}.json").read().strip().splitlines()[-1])
    cb = d.get("cpu_baseline") or {}
    print(c, "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "frac %.4f" % d["roofline"]["frac"], "cpu", cb.get("value"), cb.get("cores"))
PY
