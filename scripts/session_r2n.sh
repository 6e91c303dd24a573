set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py tests/test_gpu_ensemble.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" nolock8 noorder; do MR_ENGINE_LIB=$v BS="768" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/r2n_bs.txt 2>&1; rc=$?; echo "variant [$v] $(grep -v amdgpu.ids $OUT/r2n_bs.txt)"; [ $rc -eq 0 ] || exit $rc; done; done
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/r2n_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2n_stamps.txt; exit $rc
