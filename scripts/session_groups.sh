set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in "" g2 g8; do
  echo "variant=${v:-g4}"
  MR_ENGINE_LIB=$v BS="512" timeout -k 10 200 python scripts/c2_bs_sweep.py ibm > $OUT/grp_$v.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/grp_$v.log; [ $rc -eq 0 ] || exit $rc
  MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_c3_$v.json 2>/dev/null; rc=$?; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c3_$v.json; [ $rc -eq 0 ] || exit $rc
done
