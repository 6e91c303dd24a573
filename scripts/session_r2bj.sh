#!/bin/bash
# rehearsal of the C4 2-D layout (2 song shards cut at whole tiles x 2 user blocks) as 4 ranks on ONE GPU over
# gloo: the N > 1 bench path end to end (timing meaningless: the ranks share the GPU)
set -o pipefail
OUT=gpurun_out/r2bj; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MR_BENCH_BACKEND=gloo MR_BENCH_DEVICE=0 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --config c4 --shard 2d --song-groups 2 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/rehearsal_c4_2d4.json 2> $OUT/rehearsal_c4_2d4.err; rc=$?; echo "rehearsal rc=$rc"; grep '^{' $OUT/rehearsal_c4_2d4.json | cut -c1-700; exit $rc
