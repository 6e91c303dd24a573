#!/bin/bash
# C2 phase stamps of the final fused kernel (diagnostic build libmr_engine_stamps.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/r2bn; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 200 python scripts/stamps.py c2 ibm 0 auto > $OUT/phase_stamps_c2.txt 2>&1; rc=$?; grep -v amdgpu.ids $OUT/phase_stamps_c2.txt; exit $rc
