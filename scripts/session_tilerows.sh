set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in "" t8 t32; do
  echo "variant=${v:-t16}"
  MR_ENGINE_LIB=$v BS="512 768" timeout -k 10 200 python scripts/c2_bs_sweep.py ibm > $OUT/tr_$v.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/tr_$v.log; [ $rc -eq 0 ] || exit $rc
done
MR_ENGINE_LIB=t32 FILES="tests/test_gpu_parity.py" bash scripts/session_tests.sh
