set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
MR_WIDE_MAP=2 FILES="tests/test_gpu_parity.py" bash scripts/session_tests.sh || exit $?
timeout -k 10 400 python scripts/c4_probe.py 704 > $OUT/r2h_probe_warm.json 2>&1; rc=$?; tail -1 $OUT/r2h_probe_warm.json; [ $rc -eq 0 ] || exit $rc
for m in 1 2 1 2; do MR_WIDE_MAP=$m timeout -k 10 300 python scripts/c4_probe.py 704 > $OUT/r2h_probe_$m.json 2>&1; rc=$?; echo "map $m"; tail -1 $OUT/r2h_probe_$m.json | cut -c1-200; [ $rc -eq 0 ] || exit $rc; done
MR_WIDE_MAP=2 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc_r2h_map2_FETCH -o p -- python3 scripts/c4_probe.py 704 > $OUT/pmc_r2h.log 2>&1; rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
MR_WIDE_MAP=2 timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/pmc_r2h_map2_TCC -o p -- python3 scripts/c4_probe.py 704 > $OUT/pmc_r2h2.log 2>&1; rc=$?; echo "pmc2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python scripts/pmc_summary.py k_score_wide $OUT/pmc_r2h_map2_* 
