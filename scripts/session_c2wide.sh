set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2wide -o p -- python3 bench.py --no-cpu-baseline --stage1 wide --steps 100 > $OUT/prof_c2wide.log 2>&1; rc=$?; echo "prof rc=$rc"; cut -c1-160 $OUT/prof_c2wide/p_kernel_stats.csv; [ $rc -eq 0 ] || exit $rc
CONFIG=c2 STAGE1=wide DENSE=1 timeout -k 10 120 python scripts/large_stamps.py 0 0 ibm 2>&1 | grep -v amdgpu.ids | head -20
