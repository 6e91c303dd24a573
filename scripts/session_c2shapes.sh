set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1
for s in ${SHAPES:-fused wide separate pull user}; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --stage1 $s --steps 200 --warmup 20 > $OUT/c2_$s.json 2> $OUT/c2_$s.err; rc=$?
  echo "$s rc=$rc"; [ $rc -eq 0 ] || { tail -5 $OUT/c2_$s.err; exit $rc; }
  python -c "import json; d=json.load(open('$OUT/c2_$s.json')); print('$s', d['ms_per_step']*1000, 'us', d['launch'])"
done
