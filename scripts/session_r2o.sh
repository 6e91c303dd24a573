set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py tests/test_gpu_ensemble.py tests/test_group.py tests/test_driver.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" nosorted; do MR_ENGINE_LIB=$v BS="512 768 1024" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/r2o_bs.txt 2>&1; rc=$?; echo "variant [$v]"; grep -v amdgpu.ids $OUT/r2o_bs.txt; [ $rc -eq 0 ] || exit $rc; done; done
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/r2o_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2o_stamps.txt | head -20; exit $rc
