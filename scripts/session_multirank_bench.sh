set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 MR_BENCH_BACKEND=gloo MR_BENCH_DEVICE=0
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517"
timeout -k 10 300 $R bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline > $OUT/mr_users.json 2> $OUT/mr_users.err; rc=$?; echo "users rc=$rc"; tail -1 $OUT/mr_users.json | cut -c1-300; [ $rc -eq 0 ] || { tail -20 $OUT/mr_users.err; exit $rc; }
timeout -k 10 300 $R bench.py --gpus 2 --steps 50 --warmup 5 --no-cpu-baseline --shard songs > $OUT/mr_songs.json 2> $OUT/mr_songs.err; rc=$?; echo "songs rc=$rc"; tail -1 $OUT/mr_songs.json | cut -c1-300; [ $rc -eq 0 ] || { tail -20 $OUT/mr_songs.err; exit $rc; }
timeout -k 10 600 $R bench.py --gpus 2 --config c5 --steps 1 --warmup 0 --no-cpu-baseline > $OUT/mr_c5.json 2> $OUT/mr_c5.err; rc=$?; echo "c5 rc=$rc"; tail -1 $OUT/mr_c5.json | cut -c1-600; [ $rc -eq 0 ] || { tail -20 $OUT/mr_c5.err; exit $rc; }
