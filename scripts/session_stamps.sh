set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for a in "$@"; do
  timeout -k 10 400 python scripts/large_stamps.py $a > gpurun_out/stamps.log 2>&1; rc=$?; cat gpurun_out/stamps.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
