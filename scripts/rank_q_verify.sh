#!/bin/bash
# Verification of the fused survivor-rank threshold change (s48): the whole
# -m gpu suite, smoke, the default bench, the C1 bench, the driver's 20-step
# command, then the wide kernels' threshold (variant wq64) against production
# on C3 and C4 (kernels only).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
STEPS=tests,smoke,bench bash scripts/gpu_session.sh || exit $?
grep -q "passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "gpu suite failed"; exit 1; }
timeout -k 10 300 python bench.py --config c1 --model ubm --no-north-star --steps 200 --warmup 20 > $O/bench_c1.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-north-star > $O/bench_k20.log 2>&1 || exit 5
for v in prod wq64; do
  lib=$v; [ "$v" = prod ] && lib=""
  MR_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-e2e --no-north-star --steps 20 --warmup 3 > $O/c3_$v.log 2>&1 || exit 6
  MR_ENGINE_LIB=$lib timeout -k 10 600 python -u bench.py --config c4 --no-cpu-baseline --no-e2e --no-north-star --steps 5 --warmup 2 > $O/c4_$v.log 2>&1 || exit 7
  echo "$v c3 $(grep -o '"ms_per_step": [0-9.e-]*' $O/c3_$v.log | head -1) c4 $(grep -o '"ms_per_step": [0-9.e-]*' $O/c4_$v.log | head -1)"
done
