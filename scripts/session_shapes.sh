set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for sh in pull wide separate; do
  timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --steps 10 --warmup 2 --stage1 $sh > gpurun_out/c3_$sh.json 2>/dev/null; rc=$?
  echo "c3 $sh rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/c3_$sh.json'));print(round(d['ms_per_step'],3),'ms', d['launch'])")"
done
BS=0 bash scripts/session_variants.sh base
