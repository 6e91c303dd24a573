#!/bin/bash
# sorted-list rank merge (default) vs threshold-select merge (MR_MERGE_THRESHOLD): parity, A/B, stamps
set -o pipefail
OUT=gpurun_out/r2v; mkdir -p $OUT
K="" FILES="tests/test_gpu_parity.py tests/test_gpu_handoff.py tests/test_gpu_graph.py tests/test_api_mirror.py" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" mthr; do MR_ENGINE_LIB=$v BS="768" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/bs.txt 2>&1; rc=$?; echo "variant [$v] $(grep -v amdgpu.ids $OUT/bs.txt)"; [ $rc -eq 0 ] || exit $rc; done; done
for v in "" mthr; do MR_ENGINE_LIB=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --steps 2000 > $OUT/c2_$v.json || exit 1; echo "bench [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2_$v.json)"; done
for v in "" mthr; do MR_ENGINE_LIB=$v timeout -k 10 200 python -u bench.py --config c1 --model ubm --no-cpu-baseline --no-e2e --steps 2000 > $OUT/c1_$v.json || exit 1; echo "bench c1 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1_$v.json)"; done
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/stamps.txt; exit $rc
