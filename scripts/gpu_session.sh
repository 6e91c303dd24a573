#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace stats.
# Each GPU step has its own time limit; a crash/abort/timeout ends the session
# (test assertion failures, exit 1, do not).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-tests,smoke,bench,prof}

run() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/session.log"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/session.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name: stopping" | tee -a "$OUT/session.log"; exit $rc; fi
  # a GPU memory fault surfaces as failed tests (rc 1): stop there too
  if grep -q -E "illegal memory access|Memory access fault|HSA_STATUS_ERROR" "$OUT/$name.log"; then
    echo "GPU fault in $name: stopping" | tee -a "$OUT/session.log"; exit 86
  fi
  return $rc
}

rocminfo 2>/dev/null | grep -m1 -E "gfx950" > "$OUT/gpu.txt" || true
# targeted tests first: TESTK="expr" (pytest -k), e.g. after a kernel change
case ",$STEPS," in *,testk,*) run pytest_k 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "$TESTK" ;; esac
case ",$STEPS," in *,tests,*) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread ;; esac
case ",$STEPS," in *,smoke,*) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;; esac
# C2 headline only (no north_star / e2e / CPU baseline): kernel A/B loops
case ",$STEPS," in *,quick,*) run bench_quick 300 python bench.py --no-north-star --no-e2e --no-cpu-baseline --steps 2000 --warmup 50 ;; esac
# The driver's command (--steps 20 --warmup 5) with the K steps split into
# graphs of G steps (0 = one graph): GSTEPS="0 10 5 4 2 1", 3 runs each
case ",$STEPS," in *,k20,*)
  for gs in ${GSTEPS:-0 10 5 4 2 1}; do
    for rep in 1 2 3; do
      run k20_g${gs}_$rep 300 python bench.py --steps 20 --warmup 5 --graph-steps $gs --no-north-star --no-e2e --no-cpu-baseline
    done
  done
  run k20_nograph 300 python bench.py --steps 20 --warmup 5 --no-graph --no-north-star --no-e2e --no-cpu-baseline ;;
esac
# closing the timed region: one device-wide synchronize vs engine-stream waits first
case ",$STEPS," in *,k20sync,*)
  for rep in 1 2 3 4; do
    run k20_dev_$rep 300 python bench.py --steps 20 --warmup 5 --no-north-star --no-e2e --no-cpu-baseline
    run k20_stream_$rep 300 python bench.py --steps 20 --warmup 5 --stream-sync --no-north-star --no-e2e --no-cpu-baseline
  done ;;
esac
# host wait mode of the runtime's synchronisations: ROC_ACTIVE_WAIT_TIMEOUT (us of
# active polling before an interrupt wait), WAITS="unset 100 1000 10000"
case ",$STEPS," in *,k20wait,*)
  for wv in ${WAITS:-unset 100 1000 10000}; do
    for rep in 1 2 3; do
      if [ "$wv" = unset ]; then
        run k20_w${wv}_$rep 300 python bench.py --steps 20 --warmup 5 --no-north-star --no-e2e --no-cpu-baseline
      else
        ROC_ACTIVE_WAIT_TIMEOUT=$wv run k20_w${wv}_$rep 300 python bench.py --steps 20 --warmup 5 --no-north-star --no-e2e --no-cpu-baseline
      fi
    done
  done ;;
esac
# per-workgroup phase stamps of the scoring kernel (diagnostic build): STAMPS="c2 ibm 0 auto"
# C2 kernel A/B over library variants (scripts/build_variant.py) and engine options
# (space-separated label:key=value,... specs): VARIANTS="prod notile" OPTS="bitmap: walk:stage1_bitmap=0"
case ",$STEPS," in *,ab,*)
  for v in ${VARIANTS:-prod}; do
    lib=$v; [ "$v" = prod ] && lib=""
    MR_ENGINE_LIB=$lib run ab_$v 300 python scripts/c2_ab.py ${OPTS:-base:}
  done ;;
esac
case ",$STEPS," in *,stamps,*) run stamps 300 python scripts/stamps.py ${STAMPS:-c2 ibm 0 auto} ;; esac
case ",$STEPS," in *,ingest,*) MR_INGEST_TRACE=1 MR_LOAD_TRACE=1 run ingest_c4 900 python -u scripts/ingest_probe.py --config c4 --load --reps 3 --out "$OUT/ingest_c4.json" ;; esac
case ",$STEPS," in *,bench,*) run bench 600 python bench.py ;; esac
case ",$STEPS," in *,prof,*)
  export TMPDIR=/tmp
  run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 200 ;;
esac
case ",$STEPS," in *,c4,*) run bench_c4 900 python -u bench.py --config c4 --steps 5 --warmup 2 ;; esac
case ",$STEPS," in *,c5,*) run bench_c5 900 python -u bench.py --config c5 --steps 3 --warmup 1 ;; esac
# C5 per-model layouts (sharding.EnsembleScorer): every rank's slice on this GPU (C5N="8 4 2")
case ",$STEPS," in *,c5models,*) run c5_models 900 python -u scripts/c5_layout_probe.py ${C5N:-8} ;; esac
case ",$STEPS," in *,profc5models,*)
  export TMPDIR=/tmp
  run prof_c5_models 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c5_models" -o p -- python3 "$ROOT/scripts/c5_layout_probe.py" ${C5N:-8} ;;
esac
# the driver's C5 command at N ranks over gloo on this one GPU (per-model layouts, the all-to-all through the host)
case ",$STEPS," in *,c5rehearse,*)
  MR_BENCH_BACKEND=gloo MR_BENCH_DEVICE=0 PYTHONUNBUFFERED=1 run c5_rehearse_n2 900 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 bench.py --gpus 2 --config c5 \
    --steps 2 --warmup 1 --no-cpu-baseline ;;
esac
# C4 per ItemBasedModel route (mr_options.ibm_route): ROUTES="cooc two_hop", kernels only
case ",$STEPS," in *,c4route,*)
  for r in ${ROUTES:-cooc two_hop}; do
    run bench_c4_$r 900 python -u bench.py --config c4 --steps 5 --warmup 2 --no-e2e --no-cpu-baseline --no-north-star --ibm-route $r
  done ;;
esac
# C4 ibm over library variants (scripts/build_variant.py): VARIANTS="prod u2 u8"
case ",$STEPS," in *,c4var,*)
  for v in ${VARIANTS:-prod}; do
    lib=$v; [ "$v" = prod ] && lib=""
    export TMPDIR=/tmp
    MR_ENGINE_LIB=$lib run c4var_$v 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4var_$v" -o p -- python3 "$ROOT/bench.py" --config c4 --steps 5 --warmup 2 --no-e2e --no-cpu-baseline --no-north-star
  done ;;
esac
# phase stamps of the wide / co-listening scoring kernel: LSTAMPS="1009318 2000 ibm"
# build-phase stamps (light rows per tier, heavy-row workgroups): C4 1x1 and the 8x1 shard 0
case ",$STEPS," in *,bstamps,*)
  for lib in ${BSTAMPS_LIBS:-stamps}; do
    MR_ENGINE_LIB=$lib run bstamps_${lib}_1x1 600 python -u scripts/cooc_build_stamps.py
    SHARD=0/8 MR_ENGINE_LIB=$lib run bstamps_${lib}_8x1 600 python -u scripts/cooc_build_stamps.py
  done ;;
esac
# scoring-kernel phase stamps of the 8x1 shard 0 and of C4 1x1 (co-listening route)
case ",$STEPS," in *,sstamps,*)
  SHARD=0/8 run sstamps_8x1 600 python -u scripts/large_stamps.py 1009318 10000 ibm
  run sstamps_1x1 600 python -u scripts/large_stamps.py 1009318 10000 ibm ;;
esac
case ",$STEPS," in *,cstamps,*) run cstamps 600 python -u scripts/cooc_stamps.py ${CSTAMPS:-} ;; esac
case ",$STEPS," in *,lstamps,*) run lstamps 600 python -u scripts/large_stamps.py ${LSTAMPS:-1009318 2000 ibm} ;; esac
# C4 ibm per wide-kernel block map (MR_WIDE_MAP): MAPS="1 2 3"
case ",$STEPS," in *,c4map,*)
  export TMPDIR=/tmp
  for m in ${MAPS:-1 2 3}; do
    MR_WIDE_MAP=$m run c4map_$m 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c4map_$m" -o p -- python3 "$ROOT/bench.py" --config c4 --steps 5 --warmup 2 --no-e2e --no-cpu-baseline --no-north-star
  done ;;
esac
# any config per ibm route under rocprofv3 stats: CFG=c3 ROUTES="cooc two_hop"
case ",$STEPS," in *,cfgroute,*)
  export TMPDIR=/tmp
  for r in ${ROUTES:-cooc two_hop}; do
    run ${CFG}_$r 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${CFG}_$r" -o p -- python3 "$ROOT/bench.py" --config $CFG --steps ${CSTEPS:-20} --warmup 3 --no-e2e --no-cpu-baseline --no-north-star --ibm-route $r
  done ;;
esac
# per-rank device time of C4 layouts, one rank at a time on this GPU: LAYOUTS="1x1,2x1,4x1,8x1"
case ",$STEPS," in *,layouts,*) run layouts 900 python -u scripts/layout_probe.py ibm ${LAYOUTS:-1x1,2x1,4x1,8x1,2x4} ;; esac
# layout probe under engine-option variants: PROBES="label:KEY=V,KEY2=V;label2:..." (LAYOUTS as above)
case ",$STEPS," in *,probes,*)
  IFS=';' read -ra specs <<< "${PROBES:-base:}"
  for spec in "${specs[@]}"; do
    label=${spec%%:*}; kv=${spec#*:}
    envs=()
    IFS=',' read -ra pairs <<< "$kv"
    for x in "${pairs[@]}"; do [ -n "$x" ] && envs+=("$x"); done
    run probe_$label 600 env "${envs[@]}" MR_PROBE_REPS=${REPS:-3} python -u scripts/layout_probe.py ${PMODELS:-ibm} ${LAYOUTS:-1x1,8x1}
  done ;;
esac
# C5's two dense models per rank of each layout (C5LAYOUTS), then the ubm model at
# 1x1 under each wide block mapping (C5MAPS="1 2 3", MR_WIDE_MAP)
case ",$STEPS," in *,c5probe,*)
  MR_PROBE_CONFIG=c5 MR_PROBE_DENSE=1 MR_PROBE_REPS=${REPS:-2} run c5_layouts 900 python -u scripts/layout_probe.py ubm,ibm ${C5LAYOUTS:-1x1,8x1,2x4}
  for m in ${C5MAPS:-}; do
    MR_WIDE_MAP=$m MR_PROBE_CONFIG=c5 MR_PROBE_DENSE=1 MR_PROBE_REPS=${REPS:-2} run c5_map$m 600 python -u scripts/layout_probe.py ubm 1x1
  done ;;
esac
# rocprofv3 kernel stats of C4 (1x1, co-listening route, 3 steps) under engine-option
# variants: PROFS="label:KEY=V,KEY2=V;label2:" (env set before rocprofv3, never after --)
case ",$STEPS," in *,profs,*)
  export TMPDIR=/tmp
  IFS=';' read -ra specs <<< "${PROFS:-base:}"
  for spec in "${specs[@]}"; do
    label=${spec%%:*}; kv=${spec#*:}
    envs=()
    IFS=',' read -ra pairs <<< "$kv"
    for x in "${pairs[@]}"; do [ -n "$x" ] && envs+=("$x"); done
    run prof_$label 600 env "${envs[@]}" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$label" -o p -- python3 "$ROOT/bench.py" --config ${PCFG:-c4} --no-cpu-baseline --no-e2e --no-north-star --steps 3 --warmup 1 --ibm-route cooc
  done ;;
esac
# SQ counters of every kernel of the C4 layout probe (one pass, <= 8 SQ counters):
# LDS-bound vs memory-bound per kernel (reduce with scripts/pmc_summary.py)
case ",$STEPS," in *,pmcsq,*)
  export TMPDIR=/tmp
  MR_PROBE_REPS=1 run pmcsq_a 600 timeout -s KILL 500 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d "$OUT/pmcsq_a" -o p -- python3 "$ROOT/scripts/layout_probe.py" ibm ${LAYOUTS:-8x1}
  MR_PROBE_REPS=1 run pmcsq_b 600 timeout -s KILL 500 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$OUT/pmcsq_b" -o p -- python3 "$ROOT/scripts/layout_probe.py" ibm ${LAYOUTS:-8x1} ;;
esac
case ",$STEPS," in *,proflayouts,*)
  export TMPDIR=/tmp
  run prof_layouts 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_layouts" -o p -- python3 "$ROOT/scripts/layout_probe.py" ibm ${LAYOUTS:-8x1} ;;
esac
case ",$STEPS," in *,profc4cooc,*)
  export TMPDIR=/tmp
  run prof_c4_cooc 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4_cooc" -o bench -- python3 "$ROOT/bench.py" --config c4 --no-cpu-baseline --no-e2e --no-north-star --steps 3 --warmup 1 --ibm-route cooc ;;
esac
# Rehearsal of the driver's N>1 command on one GPU (gloo, every rank on device 0;
# the real runs use RCCL, one GPU per rank): the C2 line + its north_star block.
for n in 2 4 8; do
  case ",$STEPS," in *,rehearse$n,*)
    MR_BENCH_BACKEND=gloo MR_BENCH_DEVICE=0 PYTHONUNBUFFERED=1 run rehearse_n$n 900 python -m torch.distributed.run \
      --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n \
      --steps 50 --warmup 5 --no-cpu-baseline ;;
  esac
done
case ",$STEPS," in *,c3,*) run bench_c3 600 python bench.py --config c3 --no-cpu-baseline --steps 20 --warmup 3 ;; esac
case ",$STEPS," in *,profc3,*)
  export TMPDIR=/tmp
  run prof_c3 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o bench -- python3 "$ROOT/bench.py" --config c3 --no-cpu-baseline --steps 20 --warmup 3 ;;
esac
# PMC of one C4 neighbour batch (scripts/c4_probe.py): fetched bytes, then
# instruction / wave-cycle counters, each pass its own run
case ",$STEPS," in *,pmcc4,*)
  export TMPDIR=/tmp
  run c4probe 600 python scripts/c4_probe.py
  run pmc4_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$OUT/pmc4_fetch" -o p -- python3 "$ROOT/scripts/c4_probe.py"
  run pmc4_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-trace --output-format csv -d "$OUT/pmc4_sq" -o p -- python3 "$ROOT/scripts/c4_probe.py" ;;
esac
case ",$STEPS," in *,profc4,*)
  export TMPDIR=/tmp
  run prof_c4 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c4" -o bench -- python3 "$ROOT/bench.py" --config c4 --no-cpu-baseline --no-e2e --steps 3 --warmup 1 ;;
esac
# cost inputs of a song-factorised ubm route: the ibm index's encoding counts + both models' run times
case ",$STEPS," in *,ubmcost,*) run ubm_cost 600 python -u scripts/ubm_cost.py ${UCFG:-c5} 3 ;; esac
# PMC passes of one C4 step (scripts/pmc_bulk.sh) per library variant: PMCVARS="prod urec"
case ",$STEPS," in *,pmcvar,*)
  for v in ${PMCVARS:-prod}; do
    lib=$v; [ "$v" = prod ] && lib=""
    tag=""; [ "$v" != prod ] && tag="_$v"
    MR_ENGINE_LIB=$lib TAG=$tag run pmcvar_$v 1500 bash scripts/pmc_bulk.sh
  done ;;
esac
case ",$STEPS," in *,d2h,*) run d2h 300 python scripts/d2h_probe.py c3 3 ;; esac
exit 0
