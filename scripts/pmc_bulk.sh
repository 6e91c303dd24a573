#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit/miss; each its own rocprofv3 run,
# kernel-trace only) of one bulk-config bench command: CFG=c4|c5 (default c4),
# 1 warmup + 1 timed step; reduce with
#   IBM_ROUTE=<route> python scripts/pmc_traffic.py CFG "step:2:k_sbound" OUT.json gpurun_out/pmc_CFG_*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$(pwd)/gpurun_out; mkdir -p "$OUT"; export TMPDIR=/tmp
CFG=${CFG:-c4}
T=${CFG}${TAG:-}  # TAG: output-name suffix of a variant (e.g. MR_ENGINE_LIB=x TAG=_x)
B="$(pwd)/bench.py --config $CFG --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --no-north-star"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_${T}_fetch" -o p -- python3 $B > "$OUT/pmc_${T}_fetch.log" 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_${T}_write" -o p -- python3 $B > "$OUT/pmc_${T}_write.log" 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$OUT/pmc_${T}_tcc" -o p -- python3 $B > "$OUT/pmc_${T}_tcc.log" 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_${T}" -o p -- python3 $B > "$OUT/prof_${T}.log" 2>&1 || exit 1
