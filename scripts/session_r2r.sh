set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py tests/test_group.py" K="wide or c3" bash scripts/session_tests.sh || exit $?
timeout -k 10 400 python scripts/c4_probe.py 704 > $OUT/r2r_warm.json 2>&1; rc=$?; tail -1 $OUT/r2r_warm.json | cut -c1-150; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for f in 1 0; do MR_WIDE_FLAT=$f timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/r2r_$f.json 2>&1; rc=$?; echo "[flat=$f] $(tail -1 $OUT/r2r_$f.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
for f in 1 0; do MR_WIDE_FLAT=$f timeout -k 10 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $OUT/r2r_c3_$f.json 2>&1; rc=$?; echo "c3 flat=$f $(grep -o '"ms_per_step": [0-9.]*' $OUT/r2r_c3_$f.json)"; [ $rc -eq 0 ] || exit $rc; done
