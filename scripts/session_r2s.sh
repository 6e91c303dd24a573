set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python scripts/c4_probe.py 704 > $OUT/r2s_warm.json 2>&1; rc=$?; tail -1 $OUT/r2s_warm.json | cut -c1-150; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for cfg in "prev 1" "x 1" "x 0"; do set -- $cfg; lib=$1; [ "$lib" = x ] && lib=""; MR_ENGINE_LIB=$lib MR_WIDE_FLAT=$2 timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/r2s.json 2>&1; rc=$?; echo "[lib=$1 flat=$2] $(tail -1 $OUT/r2s.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
for cfg in "prev 1" "x 1" "x 0"; do set -- $cfg; lib=$1; [ "$lib" = x ] && lib=""; MR_ENGINE_LIB=$lib MR_WIDE_FLAT=$2 timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/r2s_c3.json 2>&1; rc=$?; echo "c3 [lib=$1 flat=$2] $(grep -o '"ms_per_step": [0-9.]*' $OUT/r2s_c3.json)"; [ $rc -eq 0 ] || exit $rc; done
