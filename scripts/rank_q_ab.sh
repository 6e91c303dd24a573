#!/bin/bash
# A/B of the survivor-rank fallback threshold (MR_RANK_Q variants built by
# scripts/build_variant.py): parity on each variant, then C1 (ubm) and C2 (ibm)
# device time per step, variants interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${RQ_VARIANTS:-q64 q256}; do
  MR_ENGINE_LIB=$v timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread \
    -k "parity or fused or topk or cand or tie or handoff" > gpurun_out/pytest_$v.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_$v.log; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for cfg in "c1 ubm" "c2 ibm"; do
    set -- $cfg
    for v in prod ${RQ_VARIANTS:-q64 q256}; do
      lib=$v; [ "$v" = prod ] && lib=""
      MR_ENGINE_LIB=$lib timeout -k 10 200 python scripts/c2_ab.py --config $1 --model $2 base: > gpurun_out/ab_${1}_${v}_$rep.log 2>&1 || exit 3
      echo "$1 $v: $(grep us_per_step gpurun_out/ab_${1}_${v}_$rep.log)"
    done
  done
done
