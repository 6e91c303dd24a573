#!/bin/bash
# Re-check of s48's outliers: the driver's 20-step command x 3, then C4 with the
# wide threshold at 16 (production) and 64 (variant wq64), interleaved twice.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out; mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-north-star --no-cpu-baseline --no-e2e > $O/k20_$rep.log 2>&1 || exit 5
  echo "k20 $rep $(grep -o '"ms_per_step": [0-9.e-]*' $O/k20_$rep.log | head -1)"
done
for rep in 1 2; do
  for v in prod wq64; do
    lib=$v; [ "$v" = prod ] && lib=""
    MR_ENGINE_LIB=$lib timeout -k 10 600 python -u bench.py --config c4 --no-cpu-baseline --no-e2e --no-north-star --steps 5 --warmup 2 > $O/c4_${v}_$rep.log 2>&1 || exit 7
    echo "$v c4 $rep $(grep -o '"ms_per_step": [0-9.e-]*' $O/c4_${v}_$rep.log | head -1)"
  done
done
