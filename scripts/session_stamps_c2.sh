set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for a in "c2 ibm 0 auto" "c2 ibm 512 fused" "c2 ibm 0 user"; do
  timeout -k 10 200 python scripts/stamps.py $a > $OUT/stamps.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/stamps.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c5.json; exit $rc
