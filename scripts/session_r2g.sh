set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/calib -o c -- ./scripts/ubench/fetch_calib > $OUT/calib.log 2>&1; rc=$?; echo "calib rc=$rc"; [ $rc -eq 0 ] || exit $rc
MR_PROBE_BYTES=1 timeout -k 10 400 python scripts/c4_probe.py 704 > $OUT/c4_probe.json 2> $OUT/c4_probe.err; rc=$?; echo "probe rc=$rc"; cat $OUT/c4_probe.json; [ $rc -eq 0 ] || exit $rc
for pass in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  tag=$(echo $pass | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pmc_r2_c4_$tag -o p -- python3 scripts/c4_probe.py 704 > $OUT/pmc_r2_c4_$tag.log 2>&1; rc=$?; echo "pmc $tag rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py k_score_wide $OUT/pmc_r2_c4_* > $OUT/pmc_r2_c4_score_wide.json; cat $OUT/pmc_r2_c4_score_wide.json
python scripts/pmc_summary.py k_neighbours $OUT/pmc_r2_c4_* > $OUT/pmc_r2_c4_neighbours.json; cat $OUT/pmc_r2_c4_neighbours.json
for k in stream16 "strided<unsigned short>" "strided<unsigned int>" "strided<unsigned long long>"; do python scripts/pmc_summary.py "$k" $OUT/calib; done > $OUT/calib_summary.txt 2>&1; cat $OUT/calib_summary.txt
find $OUT/calib -name "*counter_collection.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-40 {} | head -3' 
