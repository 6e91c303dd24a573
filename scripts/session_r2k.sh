set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py" bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/r2k_bs.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2k_bs.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/c2_bs_sweep.py ubm > $OUT/r2k_bs_ubm.txt 2>&1; rc=$?; echo ubm; grep -v amdgpu.ids $OUT/r2k_bs_ubm.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 user > $OUT/r2k_stamps_user.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2k_stamps_user.txt | head -12; exit $rc
