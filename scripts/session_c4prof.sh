set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4b -o p -- python3 scripts/large_probe.py 1009318 1000 ibm > $OUT/prof_c4b.log 2>&1; rc=$?; echo "prof rc=$rc"; grep -E "run 2|exact" $OUT/prof_c4b.log; cat $OUT/prof_c4b/p_kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/large_stamps.py 1009318 512 ibm > $OUT/stamps_c4b.txt 2>&1; rc=$?; grep -v amdgpu $OUT/stamps_c4b.txt | head -12; exit $rc
