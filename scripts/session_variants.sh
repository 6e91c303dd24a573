set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
N=${N:-"1009318 1000"}
for v in "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=$v; fi
  MR_ENGINE_LIB=$lib timeout -k 10 300 python scripts/large_probe.py $N ibm ${BS:-0} > gpurun_out/var_$v.log 2>&1; rc=$?; echo "== $v bs=${BS:-0}: $(grep -E "run 2" gpurun_out/var_$v.log) $(grep -c "exact True" gpurun_out/var_$v.log) exact"
done
