set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for r in 16 64; do
  MR_MERGE_ROWS=$r timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "parity or fused or handoff or topk" > gpurun_out/pytest_rows$r.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_rows$r.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for r in 32 16 64; do
    MR_MERGE_ROWS=$r timeout -k 10 200 python scripts/c2_ab.py base: > gpurun_out/ab_rows${r}_$rep.log 2>&1 || exit 3
    echo "rows $r: $(grep us_per_step gpurun_out/ab_rows${r}_$rep.log)"
  done
done
