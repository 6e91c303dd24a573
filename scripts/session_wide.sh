set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 > $OUT/bench_c3.json 2>/dev/null; rc=$?; echo "bench c3 rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c3.json; [ $rc -eq 0 ] || exit $rc
CONFIG=c3 DENSE=1 timeout -k 10 300 python scripts/large_stamps.py 0 0 ibm > $OUT/c3_stamps.log 2>&1; rc=$?; grep -v amdgpu.ids $OUT/c3_stamps.log | head -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c4 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/bench_c4.json 2> $OUT/bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c4.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline --steps 3 --warmup 2 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c5.json; exit $rc
