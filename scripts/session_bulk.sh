set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 python bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/bench_c5.json 2> gpurun_out/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; cat gpurun_out/bench_c5.json; tail -3 gpurun_out/bench_c5.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; cat gpurun_out/bench_c4.json; exit $rc
