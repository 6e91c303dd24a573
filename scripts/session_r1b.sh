set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 env MR_ENGINE_LIB=checks python scripts/pull_checks.py > gpurun_out/pull_checks.log 2>&1; rc=$?; echo "pull_checks rc=$rc"; tail -20 gpurun_out/pull_checks.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err; rc=$?; echo "bench c3 rc=$rc"; cat gpurun_out/bench_c3.json
