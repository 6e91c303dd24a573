set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1
bash scripts/session_tests.sh || exit $?
for c in c2 c3; do
  timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --steps 50 --warmup 5 > $OUT/bench_$c.json 2> $OUT/bench_$c.err; rc=$?; echo "bench $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json; d=json.load(open('$OUT/bench_$c.json')); print('$c', d['ms_per_step'], d['value'], d['launch'])"
done
timeout -k 10 600 python bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $OUT/bench_c5.json 2> $OUT/bench_c5.err; rc=$?; echo "bench c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "import json; d=json.load(open('$OUT/bench_c5.json')); print('c5', d['ms_per_step'], d['value'], d['threshold_mAP'])"
