set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in exp4 exp5 exp6; do
  echo "== $v"
  MR_ENGINE_LIB=$v timeout -k 10 300 python scripts/large_stamps.py 1009318 256 ibm > gpurun_out/exp_$v.log 2>&1; rc=$?; grep -E "span|stage2|user   (64|96) " gpurun_out/exp_$v.log; [ $rc -eq 0 ] || exit $rc
done
