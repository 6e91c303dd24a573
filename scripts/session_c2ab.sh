set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for lib in old ""; do
  MR_ENGINE_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/c2ab_$lib.json 2>/dev/null; rc=$?; echo "lib=${lib:-new} rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/c2ab_$lib.json'));print(d['value'], d['roofline']['avg_launch_us'])")"; [ $rc -eq 0 ] || exit $rc
done
for lib in stampsold stamps; do
  MR_ENGINE_LIB=$lib timeout -k 10 300 python scripts/stamps.py c2 ibm > gpurun_out/stamps_$lib.txt 2>&1; rc=$?; echo "== $lib"; grep -v amdgpu gpurun_out/stamps_$lib.txt; [ $rc -eq 0 ] || exit $rc
done
