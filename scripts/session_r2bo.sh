#!/bin/bash
# the driver's N > 1 command shape rehearsed on one GPU: 2 ranks over gloo, default config (C2 users shard, graph)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2bo; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MR_BENCH_BACKEND=gloo MR_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 500 --warmup 20 --no-cpu-baseline > $OUT/rehearsal_users2.json 2> $OUT/rehearsal_users2.err; rc=$?; echo "rehearsal rc=$rc"; grep '^{' $OUT/rehearsal_users2.json | cut -c1-400; exit $rc
