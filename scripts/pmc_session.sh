#!/bin/bash
# PMC counter passes (each counter group in its own rocprofv3 run, kernel-trace
# only, per MI355X_MICROARCH.md "HBM" / cdna_hip_programming.md §7), plus the
# phase-stamp diagnostics and the top-k micro-benchmark.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${CFG:-c2}
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name" >> "$OUT/pmc_session.log"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> "$OUT/pmc_session.log"
  if [ $rc -ne 0 ]; then echo "stopping: $name rc=$rc" >> "$OUT/pmc_session.log"; exit $rc; fi
}
B="$ROOT/bench.py --no-cpu-baseline --config $CFG --steps ${PSTEPS:-50} --warmup 5"
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o p -- python3 $B
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$OUT/pmc_write" -o p -- python3 $B
run pmc_tcc 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d "$OUT/pmc_tcc" -o p -- python3 $B
exit 0
