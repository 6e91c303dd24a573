set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for r in 16 32 64; do
  MR_MERGE_ROWS=$r BS="512" timeout -k 10 200 python scripts/c2_bs_sweep.py ibm > $OUT/c2_rows2_$r.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/c2_rows2_$r.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/stamps.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/stamps.log; exit $rc
