set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
bash scripts/session_tests.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/r2c_bench_c2.json 2> $OUT/r2c_bench_c2.err; rc=$?; echo "bench c2 rc=$rc"; cut -c1-300 $OUT/r2c_bench_c2.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c1 --model ubm --steps 100 --warmup 10 > $OUT/r2c_bench_c1.json 2> $OUT/r2c_bench_c1.err; rc=$?; echo "bench c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
export MR_BENCH_BACKEND=gloo MR_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --shard songs --steps 20 --warmup 3 --no-cpu-baseline > $OUT/r2c_reh_songs2.json 2> $OUT/r2c_reh_songs2.err; rc=$?; echo "rehearsal songs2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 4 --shard 2d --song-groups 2 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/r2c_reh_2d4.json 2> $OUT/r2c_reh_2d4.err; rc=$?; echo "rehearsal 2d4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
unset MR_BENCH_BACKEND MR_BENCH_DEVICE
timeout -k 10 400 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/r2c_bench_c4.json 2> $OUT/r2c_bench_c4.err; rc=$?; echo "bench c4 rc=$rc"; exit $rc
