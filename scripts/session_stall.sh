set -u
cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out; mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1; echo "list rc=$?"
grep -oE "\b(SQ|TA|TD|TCP)_[A-Z0-9_]+" $OUT/counters_list.txt | sort -u > $OUT/counter_names.txt; wc -l $OUT/counter_names.txt
P="scripts/large_probe.py 100000 1000 ibm"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/stall_sq -o p -- python3 $P > $OUT/stall_sq.log 2>&1; echo "sq rc=$?"
python scripts/pmc_summary.py k_score_wide $OUT/stall_sq > $OUT/stall_sq.json; cat $OUT/stall_sq.json
