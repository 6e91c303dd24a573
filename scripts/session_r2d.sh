set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py tests/test_api_mirror.py tests/test_jni_shim.py" bash scripts/session_tests.sh || exit $?
BS="256 512 768 1024 1536 2048" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/r2d_bs.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2d_bs.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/r2d_stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/r2d_stamps.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $OUT/r2d_bench_c2.json 2>&1; rc=$?; cut -c1-250 $OUT/r2d_bench_c2.json; exit $rc
