set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py tests/test_api_mirror.py tests/test_gpu_handoff.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2 3; do for kv in 1 0; do MR_KARG_TE_OFF=$kv BS="768" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/r2t_bs.txt 2>&1; rc=$?; echo "karg=$kv $(grep -v amdgpu.ids $OUT/r2t_bs.txt)"; [ $rc -eq 0 ] || exit $rc; done; done
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/r2t_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2t_stamps.txt | head -8; exit $rc
