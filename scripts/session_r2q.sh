set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
FILES="tests/test_gpu_parity.py" K="wide or c3" bash scripts/session_tests.sh || exit $?
timeout -k 10 400 python scripts/c4_probe.py 704 > $OUT/r2q_warm.json 2>&1; rc=$?; tail -1 $OUT/r2q_warm.json | cut -c1-150; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in "" notdel; do MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/r2q_$v.json 2>&1; rc=$?; echo "[$v] $(tail -1 $OUT/r2q_$v.json | grep -o '"device_ms": [0-9.]*')"; [ $rc -eq 0 ] || exit $rc; done; done
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_r2q_FETCH -o p -- python3 scripts/c4_probe.py 704 > $OUT/pmc_r2q.log 2>&1; rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_summary.py k_score_wide $OUT/pmc_r2q_FETCH
