#!/bin/bash
# per-wave tau in the threshold top-k (default) vs LDS-atomic row ranks (MR_NO_WAVE_TAU): all GPU tests, C2/C1/C3/C4 A/B
set -o pipefail
OUT=gpurun_out/r2af; mkdir -p $OUT
export TMPDIR=/tmp
K="" FILES="tests" bash scripts/session_tests.sh || exit $?
for rep in 1 2; do for v in "" nowtau; do MR_ENGINE_LIB=$v BS="768" timeout -k 10 300 python scripts/c2_bs_sweep.py ibm > $OUT/bs.txt 2>&1; rc=$?; echo "variant [$v] $(grep -v amdgpu.ids $OUT/bs.txt)"; [ $rc -eq 0 ] || exit $rc; done; done
for v in "" nowtau; do MR_ENGINE_LIB=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-e2e --steps 2000 > $OUT/c2_$v.json || exit 1; echo "bench c2 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c2_$v.json)"; done
for v in "" nowtau; do MR_ENGINE_LIB=$v timeout -k 10 200 python -u bench.py --config c1 --model ubm --no-cpu-baseline --no-e2e --steps 2000 > $OUT/c1_$v.json || exit 1; echo "bench c1 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c1_$v.json)"; done
for v in "" nowtau; do MR_ENGINE_LIB=$v timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/c3_$v.json 2>&1; rc=$?; echo "c3 [$v] $(grep -o '"ms_per_step": [0-9.]*' $OUT/c3_$v.json)"; [ $rc -eq 0 ] || exit $rc; done
for v in "" nowtau; do MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/c4_$v.json 2>&1; rc=$?; echo "c4 [$v] $(tail -1 $OUT/c4_$v.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/stamps.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/stamps.txt | head -16; exit $rc
