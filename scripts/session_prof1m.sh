set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_1m -o probe -- python3 scripts/large_probe.py 1009318 1000 ibm > gpurun_out/prof_1m.log 2>&1; rc=$?; tail -5 gpurun_out/prof_1m.log; find gpurun_out/prof_1m -name "*stats*" | head; cat $(find gpurun_out/prof_1m -name "*kernel_stats.csv" | head -1); exit $rc
