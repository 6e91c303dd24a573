#!/bin/bash
# Final verification of a build: the whole -m gpu suite, smoke, the default
# bench, rocprof of it, the C1 bench and the driver's 20-step command.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
STEPS=tests,smoke,bench,prof bash scripts/gpu_session.sh || exit $?
grep -q "passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log || { echo "gpu suite failed"; exit 1; }
timeout -k 10 300 python bench.py --config c1 --model ubm --no-north-star --steps 200 --warmup 20 > $O/bench_c1.log 2>&1 || exit 4
echo "c1 $(grep -o '"ms_per_step": [0-9.e-]*' $O/bench_c1.log | head -1)"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 || exit 5
echo "k20 $(grep -o '"ms_per_step": [0-9.e-]*' $O/bench_k20.log | head -2 | tr '\n' ' ')"
