set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py" bash scripts/session_tests.sh || exit $?
BS="512 768 1024" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/r2e_bs.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2e_bs.txt; [ $rc -eq 0 ] || exit $rc
for r in 16 64; do MR_MERGE_ROWS=$r BS="768" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/r2e_rows$r.txt 2>&1; rc=$?; echo "merge rows $r"; grep -v amdgpu.ids $OUT/r2e_rows$r.txt; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/r2e_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2e_stamps.txt; exit $rc
