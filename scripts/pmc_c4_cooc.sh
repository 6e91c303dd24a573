set -u
cd "${GRAFT_REPO_ROOT}"
OUT=$(pwd)/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
B="$(pwd)/bench.py --config c4 --steps 1 --warmup 1 --no-e2e --no-cpu-baseline --no-north-star"
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $OUT/pmc4c_fetch -o p -- python3 $B > $OUT/pmc4c_fetch.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/pmc4c_write -o p -- python3 $B > $OUT/pmc4c_write.log 2>&1 || exit 1
timeout -s KILL 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/pmc4c_tcc -o p -- python3 $B > $OUT/pmc4c_tcc.log 2>&1 || exit 1
