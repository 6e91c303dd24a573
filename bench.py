"""Headline benchmark: scored (test-user, song) pairs/s of the ItemBasedModel.

Workload (BASELINE.json configs[1], "C2"): ItemBasedModel over 500 train
users / 10 test users / ~16.8k songs (synthetic), 1 MI355X.
One step = one full pass of the hot path over the batch: stage 1 (neighbour
weights), stage 2 (song-tile accumulation -> every (test user, unheard song)
score written to HBM as fp32) and stage 3 (top-10 per test user) — what the
reference's getItemBasedModel computes (MusicRecommender.scala MR:222-261),
plus the recommendation list.

Multi-GPU (one process per GPU, torchrun): the headline ``value`` stays C2 at
every N (default ``--shard users``: weak scaling over test-user blocks, rank r
scores test users [10r, 10r+10) of a 500 x 10N dataset over all songs, an
exact partition of the model's pairs, no data-path collective — C2 is one
~12 us latency-bound launch, SURVEY.md §8e: "C2 is too small to scale"). The
C2 line carries a nested ``north_star`` block at every N, including 1: C4
(1M train / 10k test / 384,546 songs, top-10) in the north star's layout —
N song shards x 1 user block (sharding.ShardScorer, G_s = N: each rank the
same whole number of wide tiles, its own co-listening index over its songs;
ONE RCCL all-gather of the packed top-k record blocks per step, merged on the
device), strong scaling over the fixed test set: slowest-rank ms per step,
exchange ms, all-gather bytes, process-group sizes, the roofline of the route's
encoding-independent byte model (split per kernel, beside SURVEY.md §8(d)'s
two-hop bytes) and, at N = 1, the CPU two-hop baseline.
Rank 0 builds C4 once and the node's other ranks load its arrays.
``--shard songs`` / ``--shard 2d --song-groups G_s`` run those layouts as the
main line (``--config c4`` / ``c5`` for the full-scale configs).

Prints ONE JSON line (rank 0). See DESIGN.md §Measurement for the byte model.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (first: one HIP runtime per process)
import torch.distributed as dist  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
SCALA_PAR_PAIRS_PER_S = 508.0  # ibm par 500/10/16,785 = 330,385 ms (README.md:106)
SCALA_C1_UBM_SEQ_PAIRS_PER_S = 1120.0  # ubm seq 100/10/4,798 = 42,857 ms (README.md:72)
README_C1_MS = {"ubm": 42857, "ibm": 70839}  # README.md:72 (sequential, 100/10)
TEST_PER_GPU = 10


def _pg() -> bool:
    """A process group is up: N > 1 (torchrun), or the one-rank rehearsal of
    the collective path (MR_BENCH_PG=1). Barriers and reductions run exactly
    when this holds, so the one-rank rehearsal executes the N > 1 code."""
    return dist.is_available() and dist.is_initialized()


def algorithmic_bytes(ds, out_bytes: int = 4, k: int = 10):
    """SURVEY.md §8d byte model, split per kernel.
    Per test user u with neighbours N(u) = ∪_{s2∈T(u)} L_tr(s2):
      stage 1  12|T(u)| + 4 Σ_{s2∈T(u)} c_tr(s2)
      stage 2  Σ_{v∈N(u)} (8 + 4|S(v)|) + 4 n_s + out_bytes (n_s − |T(u)|)
      stage 3  12 k
    """
    n_s = ds.n_songs
    tr_deg = np.diff(ds.tr_off)
    trs_ptr = np.zeros(n_s + 1, dtype=np.int64)
    np.cumsum(np.bincount(ds.tr_songs, minlength=n_s), out=trs_ptr[1:])
    order = np.argsort(ds.tr_songs, kind="stable")
    trs_users = np.repeat(np.arange(ds.n_train), tr_deg)[order]
    c_tr = np.diff(trs_ptr)
    b1 = b2 = 0
    mark = np.zeros(ds.n_train, dtype=bool)
    for u in range(ds.n_test):
        T = ds.te_songs[ds.te_off[u]:ds.te_off[u + 1]]
        if T.size:
            flat = np.concatenate([trs_users[trs_ptr[s]:trs_ptr[s + 1]] for s in T])
            mark[flat] = True
            nb = np.flatnonzero(mark)
            mark[flat] = False
        else:
            nb = np.zeros(0, dtype=np.int64)
        b1 += 12 * T.size + 4 * int(c_tr[T].sum())
        b2 += int(nb.size) * 8 + 4 * int(tr_deg[nb].sum()) + 4 * n_s + out_bytes * (n_s - T.size)
    return {"neighbours": b1, "score": b2, "merge": 12 * k * ds.n_test}


def cooc_bytes(eng, ds, out_bytes: int = 4, k: int = 10):
    """Byte model of the ItemBasedModel's co-listening route,
    encoding-independent, from the engine's counts of the last ibm run
    (mr_cooc_bytes), split by kernel. Index segment (row s2, tile t) =
    min(4 nnz(s2, t), songs of t) bytes: the cheaper exact encoding (4-B
    entries or a count byte per song), whatever the build wrote.
      build_heavy  4 Σ_heavy rows (c_tr(s2) + Σ_{v∈L_tr(s2)} |S(v) ∩ shard|)   listener lists
                   and their shard rows read once (4-B ids) + the rows' index segments written
      build_light  the same over the light rows (k_cooc_light*)
      score        Σ_u Σ_{s2∈T(u)} Σ_t segment(s2, t)                        u's rows read
                   + per user 4 n_s + out_bytes (n_s − heard in the shard)  scales + dense row
      merge        12 k per user"""
    b = eng.cooc_bytes()
    n_s = eng.width
    heard = int(((ds.te_songs >= eng.song_lo) & (ds.te_songs < eng.song_hi)).sum())
    return {"build_heavy": 4 * b["heavy_reads"] + b["heavy_index_bytes"],
            "build_light": 4 * b["light_reads"] + b["light_index_bytes"],
            "score": b["consumed_bytes"] + 4 * n_s * ds.n_test + out_bytes * (n_s * ds.n_test - heard),
            "merge": 12 * k * ds.n_test}


def dataset_signature(ds):
    """Sizes identifying a generated dataset (cached byte models are keyed by it)."""
    return {"n_train": int(ds.n_train), "n_test": int(ds.n_test), "n_songs": int(ds.n_songs),
            "nnz_train": int(ds.tr_off[-1]), "nnz_test": int(ds.te_off[-1])}


def cached_twohop_bytes(cfg: str, ds):
    """SURVEY.md §8(d)'s two-hop bytes of a full-scale config, top-k only, from
    profiles/<cfg>_twohop_bytes.json (scripts/twohop_bytes.py) when its
    dataset signature matches; else None."""
    path = os.path.join(ROOT, "profiles", f"{cfg}_twohop_bytes.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    return d if d.get("signature") == dataset_signature(ds) else None


def kernel_bytes(ab, fused: bool):
    """Per-launch algorithmic bytes of the launched kernels: the fused shape
    runs all three stages in k_score; the separate shape runs stage 1 in
    k_neighbours and stages 2+3 in k_score."""
    if fused:
        return {"score": ab["neighbours"] + ab["score"] + ab["merge"]}
    return {"neighbours": ab["neighbours"], "score": ab["score"] + ab["merge"]}


def host_cores():
    """CPU threads this process can really use: the affinity mask, capped by a
    cgroup CPU quota when one is set (on the GPU box os.cpu_count() shows the
    whole machine while the job gets a share of it)."""
    n = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else n
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = max(1, min(aff, int(quota))) if quota else aff
    return {"nproc": n, "affinity": aff, "cgroup_cpu_quota": quota, "threads": usable}


def cpu_baseline(ds, model: str, seconds: float):
    """Literal restatement of getItemBasedModelP (oracle/literal.c, string ids,
    linear contains, pthreads over songs x users like MR:119-125) on all the
    host cores this job can use, timed on a bounded block of the s-major pair
    enumeration."""
    from oracle import native

    host = host_cores()
    threads = host["threads"]
    tr, te, _ = native.dataset_lines(ds)
    li = native.LiteralInputs(tr, te)
    total = ds.n_songs * ds.n_test
    n = 16 * threads
    t0 = time.perf_counter()
    li.model(model, threads=threads, pair_lo=0, pair_hi=n)
    dt = max(time.perf_counter() - t0, 1e-6)
    n = int(min(total, max(n, n * seconds / dt)))
    t0 = time.perf_counter()
    _, emitted = li.model(model, threads=threads, pair_lo=0, pair_hi=n)
    dt = time.perf_counter() - t0
    return {
        "value": emitted / dt, "unit": "pairs/s", "cores": threads, "kind": "port", "host": host,
        "sample": f"oracle/literal.c {model} (getModelP, {threads} threads): first {n} of {total} (song, user) "
                  f"pairs of the enumeration ({emitted} scored), {dt:.1f} s",
    }


def cpu_baseline_sequential(ds, model: str):
    """Config 1 is the reference's SEQUENTIAL Scala path (getUserBasedModel,
    MR:132-170, README.md:72 = 42,857 ms on an i5-8250U): the literal loop nest
    (oracle/literal.c) on one thread over the WHOLE model, timed end to end."""
    from oracle import native

    tr, te, _ = native.dataset_lines(ds)
    li = native.LiteralInputs(tr, te)
    t0 = time.perf_counter()
    _, emitted = li.model(model, threads=1)
    dt = time.perf_counter() - t0
    return {
        "value": emitted / dt, "unit": "pairs/s", "cores": 1, "kind": "port", "model_ms": dt * 1e3,
        "sample": f"oracle/literal.c {model} getModel (sequential): the whole model, {emitted} pairs, "
                  f"{dt * 1e3:.0f} ms",
        "reference_published": {"model_ms": README_C1_MS.get(model), "source": "README.md:72",
                                "hardware": "Intel i5-8250U (README.md:62), Scala 2.12 sequential"},
    }


def cpu_baseline_twohop(ds, model: str, seconds: float):
    """Full-scale configs: the literal string-id loop nest is infeasible (SURVEY.md
    §8d), so time the CPU two-hop restatement (oracle/fixedpoint.c, top-k only)
    on all the host cores this job can use: one thread per core, each over its
    own block of test users (ctypes releases the GIL), bounded to ~`seconds`."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import native

    host = host_cores()
    T = max(1, min(host["threads"], ds.n_test))

    def pairs(lo, hi):
        return (hi - lo) * ds.n_songs - int(ds.te_off[hi] - ds.te_off[lo])

    def run(n):  # n users per thread, thread t: users [t n, (t+1) n)
        blocks = [(t * n, (t + 1) * n) for t in range(T)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(T) as ex:
            list(ex.map(lambda b: native.fp_model(ds, model, user_lo=b[0], user_hi=b[1], k=10, dense=False),
                        blocks))
        return time.perf_counter() - t0, sum(pairs(*b) for b in blocks)

    # Each call re-transposes the train CSR (a fixed cost the reference's timed
    # region does not contain): rate = difference of two per-thread user counts.
    prev = None
    n = 1
    while True:
        dt, p = run(n)
        if (dt > seconds / 3 and prev is not None) or (n + 1) * T > ds.n_test:
            break
        prev = (n, dt, p)
        n = min(ds.n_test // T, n * 2)
    if prev is None:
        prev = (0, 0.0, 0)
    dp, dtt = p - prev[2], max(dt - prev[1], 1e-9)
    return {
        "value": dp / dtt, "unit": "pairs/s", "cores": T, "kind": "port", "host": host,
        "sample": f"oracle/fixedpoint.c {model} two-hop (int64 fixed point, top-10 only), {T} threads over "
                  f"disjoint test-user blocks: {n} vs {prev[0]} users per thread ({dp} more pairs) in {dtt:.1f} s "
                  f"more (difference of two runs, so the per-call train transpose is excluded)",
    }


def run_c5(args, world: int, rank: int, local: int) -> None:
    """Config 5: the reference's whole evaluation pipeline on device — ubm + ibm
    dense models, linear / aggregation / stochastic combinations (main.scala:57-89,
    MR:317-481) and the threshold mAP of all five (MR:636), 2,000 test users
    against the full train set. N > 1 (--c5-layout models, the default):
    sharding.EnsembleScorer — ubm by test-user blocks, ibm by song shards, ONE
    all-to-all of the ibm rows into the blocks, the combinations and the five
    mAPs on the blocks (one MAX + one SUM all-reduce over RCCL); --c5-layout
    grid: both models in the 2-D layout of sharding.ShardScorer (--shard)."""
    from musicrecommendation_amd import evaluation
    from musicrecommendation_amd.ensemble import DeviceEnsemble
    from musicrecommendation_amd.sharding import EnsembleScorer, layout_2d, shard_tile, song_shards, user_blocks

    n_tr, n_te, _seed = synth.BULK_CONFIGS["c5"]
    full, setup_s = shared_bulk_dataset("c5", world, rank)  # N > 1: rank 0 generates, the others load
    coll = True if _pg() else None
    if args.c5_layout == "models":
        sc = EnsembleScorer(full, rank, world, local, out_dtype="f32", ibm_route=args.ibm_route, collectives=coll)
        ens, eng, ds = sc.ens, sc.eng_i, full
        layout = f"ubm: users{world} blocks, ibm: songs{world} shards, one all-to-all" if world > 1 else "songs1xusers1"

        def step():
            return sc.step(0.5, 0.5, 0.5, seed=1)
    else:
        sc = None
        gs, gu = layout_2d(world, song_groups_for(args, world))
        a, b = user_blocks(full.n_test, gu)[rank // gs]
        lo, hi = song_shards(full, gs, shard_tile(full.n_train, full.n_test // gu, n_songs=full.n_songs,
                                                  n_shards=gs))[rank % gs]
        ds = full if gu == 1 else full.subset_test_users(a, b)
        eng = Engine(ds, device=local, out_dtype="f32", topk=10, song_lo=lo, song_hi=hi, ibm_route=args.ibm_route)
        ens = DeviceEnsemble(eng, pair_base=a * full.n_songs - int(full.te_off[a]), n_pairs=full.n_pairs(),
                             pos=evaluation.label_pos(full), n_label_songs=full.n_label_songs, collectives=coll)
        layout = f"songs{gs}xusers{gu}"

        def step():
            ubm, ibm = ens.model("ubm"), ens.model("ibm")
            # the three combinations in one pass, their min / max carried to threshold_map
            lcm, am, scm = ens.combinations(ubm, ibm, 0.5, 0.5, 0.5, seed=1)
            models = {"ubm": ubm, "ibm": ibm, "lcm": lcm, "am": am, "scm": scm}
            return models, ens.threshold_maps(models)

    models = None
    for _ in range(args.warmup):
        models = None  # release the previous step's buffers so the allocator reuses them
        models, maps = step()
    if _pg():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        models = None
        models, maps = step()
    torch.cuda.synchronize()
    if _pg():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_max = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if _pg():
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    elapsed = float(t_max.item())
    songs = None
    if world == 1:
        songs, _sc, _k = ens.topk(models["lcm"])
    if rank == 0:
        pairs = full.n_pairs()
        value = pairs * args.steps / elapsed
        ab = algorithmic_bytes(full, 4, 10)
        model_bytes = sum(ab.values())
        ibm_bytes = model_bytes
        if eng.ibm_route == "cooc":  # the ibm model's byte model on its route (counts of the last ibm run)
            ibm_bytes = sum(cooc_bytes(eng, eng.dataset, 4, 10).values())
            if world > 1:  # rank 0's song shard: the whole model's ~ N x that (shards cut equal)
                ibm_bytes *= world
        dense_elems = full.n_test * full.n_songs
        # per step: 2 models + the combinations' one pass (2 reads + 3 writes) + min/max reads of the
        # 2 models (the combinations carry theirs) + 5 counts reads
        step_bytes = model_bytes + ibm_bytes + dense_elems * 4 * (2 + 3 + 2 + 5)
        step_s = elapsed / args.steps
        traffic = None
        pmc_file = os.path.join(ROOT, "profiles", "pmc_c5.json")
        if world == 1 and os.path.exists(pmc_file):  # per-step PMC sum (scripts/pmc_traffic.py step mode)
            with open(pmc_file) as f:
                pmc = json.load(f)
            if (pmc.get("ibm_route") or "two_hop") == eng.ibm_route:  # counters of the same ibm route only
                traffic = pmc.get("traffic_bytes_per_launch")
        line = {
            "metric": "scored (test-user,song) pairs/sec, ensemble ubm+ibm+lcm+am+scm + threshold mAP",
            "value": value, "unit": "pairs/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": step_s * 1e3, "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "int64", "ibm_route": eng.ibm_route,
            "data": "synthetic (bulk Zipf/lognormal Taste-Profile-shaped triplets, capped head, SURVEY.md §8d)",
            "config": {"workload": f"c5: {n_tr} train / {n_te} test / {full.n_songs} songs; ubm + ibm dense fp32, "
                                   f"linear(0.5) + aggregation(0.5) + stochastic(0.5, seed 1), threshold mAP x5",
                       "n_train": n_tr, "n_test": n_te, "n_songs": full.n_songs, "pairs_per_step": pairs,
                       "parallelism": layout},
            "exchange_bytes_per_rank": sc.exchange_bytes if sc is not None and world > 1 else None,
            "setup_dataset_s": setup_s,
            "roofline": {"bound": "hbm", "kernel": "whole step (2 scoring passes + 3 combinations + 5 evaluations)",
                         "achieved": step_bytes / step_s / 1e9, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                         "frac": step_bytes / step_s / 1e9 / (HBM_PEAK_GBS * world), "traffic": traffic,
                         "traffic_source": "profiles/pmc_c5.json (rocprofv3 --pmc passes over one step, every "
                                           "engine kernel summed)" if traffic else None,
                         "traffic_GBps": traffic / step_s / 1e9 if traffic else None,
                         # measured fabric bytes per second over the 8 TB/s peak: how saturated the
                         # step is, whatever the byte model says (frac counts algorithmic bytes only)
                         "traffic_frac": traffic / step_s / 1e9 / HBM_PEAK_GBS if traffic else None,
                         "algorithmic_bytes_per_step": step_bytes},
            "threshold_mAP": maps,
            "mAP@10_lcm": evaluation.map_at_k(songs, full, 10) if songs is not None else None,
            "cpu_baseline": (cpu_baseline_twohop(full, "ibm", args.cpu_baseline_seconds)
                             if world == 1 and not args.no_cpu_baseline else None),
        }
        if world == 1 and not args.no_e2e:
            models = None
            if sc is not None:
                sc.close()
                sc = None
            line["end_to_end"] = end_to_end_c5(synth.config("c5"))
        print(json.dumps(line), flush=True)
    if sc is not None:
        sc.close()
    else:
        eng.close()
    if _pg():
        dist.destroy_process_group()


def end_to_end_c5(trip, reps: int = 2):
    """C5's own pipeline on one GPU, wall clock: ingest of the three TSV files
    (native reader, ≙ the MusicRecommender constructor, MR:26-91) -> mr_load
    (host index build + H2D) -> both dense models, the three combinations and
    the five threshold mAPs (main.scala:37-89 without the prints: the mAP
    values are the pipeline's output, MR:636). Median of `reps` runs; the files
    are written once beforehand (untimed)."""
    import tempfile

    from musicrecommendation_amd.dataset import Dataset
    from musicrecommendation_amd.sharding import EnsembleScorer

    rows = []
    with tempfile.TemporaryDirectory() as td:
        paths = [os.path.join(td, n) for n in ("train.txt", "test.txt", "labels.txt")]
        t0 = time.perf_counter()
        nbytes = trip.write_tsv(*paths)
        write_s = time.perf_counter() - t0
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d2 = Dataset.from_tsv(*paths)
            t1 = time.perf_counter()
            sc = EnsembleScorer(d2, 0, 1, torch.cuda.current_device(), out_dtype="f32")
            t2 = time.perf_counter()
            models, maps = sc.step(0.5, 0.5, 0.5, seed=1)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            del models
            sc.close()
            rows.append((t3 - t0, t1 - t0, t2 - t1, t3 - t2))
            del d2
    rows.sort()
    tot, ing, load, run = rows[len(rows) // 2]
    n_rows = int(trip.train_u.size + trip.test_u.size + trip.label_u.size)
    return {"ms": tot * 1e3, "rows": n_rows, "tsv_bytes": nbytes,
            "breakdown_ms": {"ingest_tsv": ing * 1e3, "mr_load_index_h2d": load * 1e3,
                             "models_combinations_5_maps": run * 1e3},
            "ingest_rows_per_s": n_rows / ing, "host_cores": host_cores()["threads"],
            "note": f"wall clock, one GPU, median of {reps}: native TSV ingest (mr_corpus_from_tsv) + mr_load + "
                    f"ubm + ibm dense models + the three combinations + the five threshold mAPs (the values the "
                    f"reference's driver prints); files written beforehand in {write_s:.1f} s (untimed)"}


def song_groups_for(args, world: int) -> int:
    """G_s of the layout: --shard songs -> world, users -> 1, 2d -> --song-groups
    (default 2 when it divides world, else world)."""
    if args.shard == "songs":
        return world
    if args.shard == "users":
        return 1
    if args.song_groups:
        return args.song_groups
    return 2 if world % 2 == 0 else world


def end_to_end(ds, model: str, reps: int = 3):
    """The reference's whole call chain on one GPU, wall clock: ingest of the
    three TSV files (native reader, ≙ the constructor MR:26-91) -> mr_load
    (host-side index build + H2D) -> mr_run -> D2H of the dense fp32 model
    (≙ getModel's result array, MR:105-111). Median of `reps` runs; the files
    are written once beforehand (untimed)."""
    import tempfile

    from musicrecommendation_amd.dataset import Dataset

    rows = []
    with tempfile.TemporaryDirectory() as td:
        paths = [os.path.join(td, n) for n in ("train.txt", "test.txt", "labels.txt")]
        ds.write_tsv(*paths)
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d2 = Dataset.from_tsv(*paths)
            t1 = time.perf_counter()
            e = Engine(d2, device=torch.cuda.current_device(), out_dtype="f32", topk=10)
            t2 = time.perf_counter()
            e.run(model)
            e.sync()
            t3 = time.perf_counter()
            dense = e.dense()
            t4 = time.perf_counter()
            e.close()
            rows.append((t4 - t0, t1 - t0, t2 - t1, t3 - t2, t4 - t3))
            d2h_bytes = int(dense.nbytes)
            del dense, d2  # freed outside the timed region (munmap of the previous rep's array)
    rows.sort()
    tot, ing, load, run, d2h = rows[len(rows) // 2]
    return {"ms": tot * 1e3, "pairs_per_s": ds.n_pairs() / tot,
            "breakdown_ms": {"ingest_tsv": ing * 1e3, "mr_load_index_h2d": load * 1e3, "mr_run": run * 1e3,
                             "d2h_dense": d2h * 1e3},
            "d2h_bytes": d2h_bytes, "d2h_GBps": d2h_bytes / d2h / 1e9,
            "note": "wall clock, one GPU: native TSV ingest + mr_load (host index build + H2D) + mr_run + "
                    "D2H of the dense fp32 model; median of 3 (value excludes all of this but the kernels)"}


def shared_bulk_dataset(cfg: str, world: int, rank: int):
    """The full-scale dataset of every rank: at N > 1 rank 0 generates it once
    (~20 s of numpy at C4) and writes its arrays to a node-local temporary
    file that the other ranks load after a barrier (one process per GPU on ONE
    node); returns (dataset, seconds)."""
    import shutil
    import tempfile

    from musicrecommendation_amd.dataset import Dataset

    t0 = time.perf_counter()
    if not _pg():
        return synth.config(cfg).dataset(), time.perf_counter() - t0
    path = [None]
    full = None
    if rank == 0:
        full = synth.config(cfg).dataset()
        d = tempfile.mkdtemp(prefix=f"mr_{cfg}_", dir=os.environ.get("TMPDIR", "/tmp"))
        full.save_arrays(os.path.join(d, "ds.npz"))
        path = [d]
    dist.broadcast_object_list(path, src=0)
    if rank != 0:
        full = Dataset.load_arrays(os.path.join(path[0], "ds.npz"))
    dist.barrier()
    if rank == 0:
        shutil.rmtree(path[0], ignore_errors=True)
    return full, time.perf_counter() - t0


def host_peak_rss_gb() -> float:
    import resource

    return resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2 ** 20  # KiB -> GiB


def north_star(args, world: int, rank: int, local: int):
    """The north star's layout at this N (BASELINE.json: "item-item similarity
    partitions by song-id range across the 8 GPUs ... with a single RCCL
    all-gather of per-test-user partial scores"): C4 = the full Taste-Profile
    shape (1,009,318 train / 10,000 test / 384,546 songs, top-10), strong
    scaling over the fixed test set: N song shards (sharding.ShardScorer with
    G_s = N, G_u = 1), each an equal whole number of tiles
    (mr_shard_tile_songs_n: C4 over 8 shards = 24 tiles, 3 per GPU); every
    rank scores all test users over its songs — with the co-listening route
    its index holds only its songs' columns, so nothing is built twice (user
    blocks would each rebuild the popular rows) — and the shards exchange
    their top-k record blocks with ONE all-gather (RCCL) and merge them on the
    device (distributed.scala:477-479's song partition). Every rank runs this;
    returns the block for rank 0's line (None elsewhere).

    Roofline: the route's encoding-independent byte model (cooc_bytes, summed
    over the ranks' shards, + the exchange's merge) over the slowest rank's
    device time per step (HIP events on each engine stream), against N x 8 TB/s;
    SURVEY.md §8(d)'s two-hop bytes beside it (profiles/c4_twohop_bytes.json).
    At N = 1 the measured traffic (profiles/pmc_c4.json, same route) and the
    CPU two-hop baseline (oracle/fixedpoint.c, the usable host cores, after the
    timed region)."""
    from musicrecommendation_amd.sharding import ShardScorer

    cfg = args.ns_config
    full, gen_s = shared_bulk_dataset(cfg, world, rank)
    gs = world
    t0 = time.perf_counter()
    scorer = ShardScorer(full, rank, world, local, song_groups=gs, topk=10, dense=False, out_dtype="f32",
                         ibm_route=args.ibm_route)
    rehearse = _pg() and world == 1  # MR_BENCH_PG=1: the one-rank group runs the exchange too
    scorer.exchange_always = rehearse
    exchanging = scorer.gs > 1 or rehearse
    load_s = time.perf_counter() - t0
    free_b, total_b = torch.cuda.mem_get_info(scorer.device)
    eng = scorer.engine

    def timed(fn, k, window=False):
        if _pg():
            dist.barrier()
        torch.cuda.synchronize()
        scorer.sync()
        t = time.perf_counter()
        if window:
            eng.timing_begin()
        for _ in range(k):
            fn()
        if window:
            eng.timing_stop()
        scorer.sync()
        torch.cuda.synchronize()
        if _pg():
            dist.barrier()
        el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device="cuda")
        if _pg():
            dist.all_reduce(el, op=dist.ReduceOp.MAX)
        return float(el.item())

    for _ in range(args.ns_warmup):
        scorer.step(args.model)
    step_s = timed(lambda: scorer.step(args.model), args.ns_steps, window=True)
    _n, win_ms = eng.timing_end()  # this rank's engine-stream time over the timed steps
    exch_s = timed(scorer.exchange, args.ns_steps) if exchanging else 0.0
    cooc = args.model == "ibm" and eng.ibm_route == "cooc"
    split = cooc_bytes(eng, scorer.ds, 0, 10) if cooc else {}
    if cooc and exchanging:  # the exchange's merge: G_s gathered lists read, one written, per user
        split["exchange_merge"] = 12 * 10 * scorer.ds.n_test * (scorer.gs + 1)  # this rank: G_s lists in, one out
    keys = ["build_heavy", "build_light", "score", "merge", "exchange_merge"]
    vec = [float(split.get(k_, 0)) for k_ in keys]
    vec += [float(scorer.pairs()), win_ms / args.ns_steps, host_peak_rss_gb(), float(total_b - free_b)]
    st = torch.tensor(vec, dtype=torch.float64, device="cuda")
    if _pg():
        sums = st.clone()
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        maxs = st.clone()
        dist.all_reduce(maxs, op=dist.ReduceOp.MAX)
        sums, maxs = sums.tolist(), maxs.tolist()
    else:
        sums = maxs = st.tolist()
    nk = len(keys)
    byte_split = {k_: int(v) for k_, v in zip(keys, sums[:nk]) if v}
    pairs, dev_ms = sums[nk], maxs[nk + 1]
    out = None
    if rank == 0:
        ms = step_s / args.ns_steps * 1e3
        step_bytes = sum(byte_split.values())
        roof = None
        if cooc and dev_ms > 0:
            ach = step_bytes / (dev_ms * 1e-3) / 1e9
            peak = HBM_PEAK_GBS * world
            traffic = traffic_src = None
            pmc_file = os.path.join(ROOT, "profiles", "pmc_c4.json")
            if world == 1 and os.path.exists(pmc_file):
                with open(pmc_file) as f:
                    pmc = json.load(f)
                if pmc.get("ibm_route") == "cooc" and pmc.get("layout", "1x1") == "1x1":
                    traffic = pmc.get("traffic_bytes_per_launch")
                    traffic_src = "profiles/pmc_c4.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, one C4 step)"
            th = cached_twohop_bytes(cfg, full)
            roof = {
                "bound": "hbm", "kernel": "whole step: k_cooc_build + k_cooc_light* + k_score_wide<cooc> + "
                                          "k_topk_merge (+ the exchange's merge at N > 1)",
                "byte_model": "co-listening route, encoding-independent: per (row, tile) segment min(4 nnz, "
                              "tile songs) B; listener lists + their shard rows read once as 4-B ids "
                              "(bench.cooc_bytes, mr_cooc_bytes), summed over the N shards",
                "achieved": ach, "peak": peak, "unit": "GB/s", "frac": ach / peak,
                "traffic": traffic, "traffic_source": traffic_src,
                "traffic_frac": traffic / (dev_ms * 1e-3) / 1e9 / peak if traffic else None,
                "algorithmic_bytes_per_step": step_bytes, "bytes_per_kernel": byte_split,
                "device_ms_per_step": dev_ms,
                "timing": "HIP events on each rank's engine stream around the timed steps; max over ranks",
                "survey_two_hop": ({"bytes_per_step": th["total_bytes"], "source": "profiles/c4_twohop_bytes.json "
                                   "(scripts/twohop_bytes.py: SURVEY.md §8(d), top-10 only)",
                                   "equivalent_GBps": th["total_bytes"] / (dev_ms * 1e-3) / 1e9,
                                   "equivalent_frac": th["total_bytes"] / (dev_ms * 1e-3) / 1e9 / peak,
                                   "note": "modelled, not measured: the survey's two-hop algorithm's bytes over "
                                           "the same time; the route computes the same integer sums without "
                                           "moving them (DESIGN.md §4b), so this may exceed 1"} if th else None),
            }
        out = {
            "workload": f"{cfg}: {'ItemBasedModel' if args.model == 'ibm' else 'UserBasedModel'} {full.n_train} train / "
                        f"{full.n_test} test / {full.n_songs} songs, top-10 only",
            "layout": f"songs{scorer.gs}xusers{scorer.gu}", "song_shards": scorer.gs, "user_blocks": scorer.gu,
            "ibm_route": eng.ibm_route, "tiles_per_rank": eng.n_tiles, "block_songs": eng.block_songs,
            "songs_per_rank": eng.width,
            "value": pairs * args.ns_steps / step_s, "unit": "pairs/s", "scaling": "strong",
            "pairs_per_step": pairs, "steps": args.ns_steps, "warmup": args.ns_warmup,
            "ms_per_step": ms,  # slowest rank: max over ranks of the barrier-bracketed window
            "device_ms_per_step": dev_ms,
            "exchange_ms_per_step": exch_s / args.ns_steps * 1e3 if exchanging else 0.0,
            "exchange": ("one all_gather_into_tensor of the top-k record blocks (int64 keys + int32 songs) per "
                         "step inside each user block, then k_topk_merge on the device" if exchanging else
                         "none (one song shard: no exchange)"),
            "allgather_bytes_per_rank": scorer.gs * scorer.rec_bytes if exchanging else 0,
            "record_bytes": scorer.rec_bytes,
            "process_group": {"backend": dist.get_backend() if _pg() else None,
                              "world_size": dist.get_world_size() if _pg() else 1,
                              "block_group_size": dist.get_world_size(scorer.group) if _pg() else 1,
                              "rehearsal": "MR_BENCH_PG=1: one-rank group, exchange forced" if rehearse else None},
            "setup_s": {"dataset": gen_s, "shard_load": load_s},
            "host": {"threads_per_rank": _usable_threads(), "peak_rss_gb_max_rank": maxs[nk + 2],
                     "peak_rss_gb_sum": sums[nk + 2], "device_used_gb_after_load_max": maxs[nk + 3] / 2 ** 30},
            "roofline": roof,
            "note": "strong scaling: the N=1 line runs the whole C4 step on one GPU; compare ms_per_step across N",
        }
    eng.close()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:  # after the timed region
        out["cpu_baseline"] = cpu_baseline_twohop(full, args.model, args.cpu_baseline_seconds)
        out["vs_cpu_baseline"] = out["value"] / out["cpu_baseline"]["value"]
    return out


def _usable_threads() -> int:
    from musicrecommendation_amd.mr_par_info import usable_cores

    return usable_cores()


def end_to_end_bulk(trip, model: str, reps: int = 2, k: int = 10):
    """Full-scale configs (C4/C5), one GPU, wall clock: the reference's whole
    call chain at the size the native ingest exists for — ingest of the three
    TSV files (48.4M rows at C4; ≙ the MusicRecommender constructor,
    MR:26-91) -> mr_load (host index build + H2D) -> mr_run -> D2H of the
    top-k lists (the dense model is 15 GB at C4: top-k output, SURVEY.md §7
    hard part 4). The files are written once beforehand (untimed)."""
    import tempfile

    from musicrecommendation_amd.dataset import Dataset

    rows = []
    with tempfile.TemporaryDirectory() as td:
        paths = [os.path.join(td, n) for n in ("train.txt", "test.txt", "labels.txt")]
        t0 = time.perf_counter()
        nbytes = trip.write_tsv(*paths)
        write_s = time.perf_counter() - t0
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            d2 = Dataset.from_tsv(*paths)
            t1 = time.perf_counter()
            e = Engine(d2, device=torch.cuda.current_device(), topk=k, dense=False)
            t2 = time.perf_counter()
            e.run(model)
            e.sync()
            t3 = time.perf_counter()
            songs, _sc, _k = e.topk()
            t4 = time.perf_counter()
            e.close()
            rows.append((t4 - t0, t1 - t0, t2 - t1, t3 - t2, t4 - t3))
            del d2
    rows.sort()
    tot, ing, load, run, d2h = rows[len(rows) // 2]
    n_rows = int(trip.train_u.size + trip.test_u.size + trip.label_u.size)
    return {"ms": tot * 1e3, "rows": n_rows, "tsv_bytes": nbytes,
            "breakdown_ms": {"ingest_tsv": ing * 1e3, "mr_load_index_h2d": load * 1e3, "mr_run": run * 1e3,
                             "d2h_topk": d2h * 1e3},
            "ingest_rows_per_s": n_rows / ing, "host_cores": host_cores()["threads"],
            "note": f"wall clock, one GPU, median of {reps}: native TSV ingest (mr_corpus_from_tsv) + mr_load + "
                    f"mr_run + D2H of the top-{k} lists; files written beforehand in {write_s:.1f} s (untimed)"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--model", default="ibm", choices=["ibm", "ubm"])
    ap.add_argument("--shard", default="users", choices=["users", "songs", "2d"],
                    help="N > 1 layout: test-user blocks (default), song-range shards + all-gather of the "
                         "top-k lists (north star), or the 2-D product of both (--song-groups)")
    ap.add_argument("--song-groups", type=int, default=0, help="2d: song shards per user block")
    ap.add_argument("--c5-layout", default="models", choices=["models", "grid"],
                    help="C5 at N > 1: each model in its own layout (ubm by user blocks, ibm by song shards, "
                         "one all-to-all; default) or both in the --shard grid")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (ingest + H2D + D2H) timing")
    ap.add_argument("--no-north-star", action="store_true",
                    help="skip the nested C4 2-D layout block (north_star) of the C2 line")
    ap.add_argument("--ns-steps", type=int, default=5, help="timed steps of the north_star block")
    ap.add_argument("--ns-warmup", type=int, default=2, help="warmup steps of the north_star block")
    ap.add_argument("--ns-config", default="c4", help="dataset of the north_star block (c4; smaller ones for "
                                                       "rehearsals of the collective path)")
    ap.add_argument("--inflight", type=int, default=1,
                    help="independent C2 batches kept in flight per GPU (own context + stream each); "
                         "steps are issued round-robin, so up to this many overlap on the device")
    ap.add_argument("--stage1", default="auto", choices=["auto", "fused", "separate", "wide"],
                    help="launch shape (default: the engine's choice)")
    ap.add_argument("--block-songs", type=int, default=0, help="songs per tile (default: the engine's choice)")
    ap.add_argument("--ibm-route", default="auto", choices=["auto", "two_hop", "cooc"],
                    help="wide shape's ItemBasedModel route (mr_options.ibm_route)")
    ap.add_argument("--graph", action=argparse.BooleanOptionalAction, default=True,
                    help="users shard, small configs: replay the K timed steps as one captured HIP graph "
                         "(--no-graph: K stream launches)")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps per captured graph (must divide --steps; 0 = all K in one graph)")
    ap.add_argument("--rehearse", action=argparse.BooleanOptionalAction, default=True,
                    help="graph path: run the timed region's call sequence once, untimed, before it")
    ap.add_argument("--stream-sync", action="store_true",
                    help="close the timed region with engine-stream waits before torch.cuda.synchronize() "
                         "(default: one device-wide synchronize, the window's event read afterwards)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="HBM bytes per score-kernel launch measured by rocprofv3 PMC (profiles/)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    # Rehearsal overrides (never set by the driver): MR_BENCH_BACKEND=gloo and
    # MR_BENCH_DEVICE=0 let several ranks share one GPU to exercise the N > 1
    # code paths on a one-GPU box; MR_BENCH_PG=1 brings the process group up at
    # N = 1 too, so the driver's N > 1 collectives (RCCL init with device_id,
    # broadcast_object_list, barriers, all-reduces, the all-gather exchange)
    # run on one GPU. The real runs use RCCL, one GPU per rank.
    backend = os.environ.get("MR_BENCH_BACKEND", "nccl")
    if "MR_BENCH_DEVICE" in os.environ:
        local = int(os.environ["MR_BENCH_DEVICE"])
    torch.cuda.set_device(local)
    if world > 1 or os.environ.get("MR_BENCH_PG") == "1":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    if args.config == "c5":
        run_c5(args, world, rank, local)
        return
    bulk = args.config in synth.BULK_CONFIGS
    if bulk:  # full-scale: fixed test set, top-k only (SURVEY.md §8d OUT = 12k)
        n_tr, n_te, _seed = synth.BULK_CONFIGS[args.config]
    else:
        n_tr, n_te, _seed, _t = synth.CONFIGS[args.config]
    dense_out = not bulk
    if args.shard == "users" and not bulk:
        # weak scaling: rank r, in-flight slot j scores test-user block
        # (r * inflight + j) of a 500 x (10 * world * inflight) dataset: disjoint
        # blocks, same train set, no data-path collective
        nb = world * args.inflight
        full = synth.config(args.config, n_test=n_te * nb).dataset()
        blocks = [full.subset_test_users(b * n_te, (b + 1) * n_te)
                  for b in range(rank * args.inflight, (rank + 1) * args.inflight)]
        engines = [Engine(b, device=local, out_dtype="f32", topk=10, stage1=args.stage1, block_songs=args.block_songs,
                          ibm_route=args.ibm_route) for b in blocks]
        ds = blocks[0]
        eng = engines[0]
        pairs_per_engine = [b.n_pairs() for b in blocks]
        step_i = [0]

        def step():
            j = step_i[0] % len(engines)
            engines[j].run(args.model)
            step_i[0] += 1

        def drain():
            for e in engines:
                e.sync()

        def rank_pairs(k):
            return float(sum(pairs_per_engine[i % len(engines)] for i in range(k)))
    else:
        # 2-D layout (sharding.ShardScorer): user blocks x song shards with one
        # all-gather of the top-k lists per block. bulk: strong scaling over the
        # fixed test set; small configs: weak, 10 test users per GPU in total.
        from musicrecommendation_amd.sharding import ShardScorer

        if bulk and _pg():  # built once on the node (rank 0), loaded by the other ranks
            trip = None
            full, _gen_s = shared_bulk_dataset(args.config, world, rank)
        else:
            trip = synth.config(args.config, n_test=None if bulk else n_te * world)
            full = trip.dataset()
        scorer = ShardScorer(full, rank, world, local, song_groups=song_groups_for(args, world), topk=10,
                             out_dtype="f32", dense=dense_out, stage1=args.stage1, block_songs=args.block_songs,
                             ibm_route=args.ibm_route)
        eng = scorer.engine
        ds = scorer.ds
        engines = [eng]
        pr = scorer.pairs()

        def step():
            scorer.step(args.model)

        def drain():
            scorer.sync()

        def rank_pairs(k):
            return float(pr) * k

    for _ in range(args.warmup):
        step()
    drain()
    if args.shard == "users" and not bulk:
        step_i[0] = 0
    use_graph = args.graph and args.shard == "users" and not bulk and args.inflight == 1
    g_steps = args.graph_steps if 0 < args.graph_steps <= args.steps and args.steps % args.graph_steps == 0 \
        else args.steps
    if use_graph:  # the K timed steps as K / G replays of a G-step HIP graph (captured untimed)
        eng.graph_capture(args.model, g_steps)
        eng.graph_launch()  # first replay uploads the graph: untimed
        drain()
    if use_graph and args.rehearse:
        # The timed region's exact call sequence once, untimed (warmup): the
        # first window's event records and closing synchronisation otherwise
        # pay their first-call cost inside the only region a short run times
        # (profiles/r06/s17-s18).
        if _pg():
            dist.barrier()
        torch.cuda.synchronize()
        eng.timing_begin()
        for _ in range(args.steps // g_steps):
            eng.graph_launch()
        eng.timing_stop()
        torch.cuda.synchronize()
        eng.timing_end()
        drain()
    if _pg():
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.timing_begin()  # HIP events on the engine's own stream, around the timed steps
    if use_graph:
        for _ in range(args.steps // g_steps):
            eng.graph_launch()
    else:
        for _ in range(args.steps):
            step()
    t_submit = time.perf_counter() - t0  # host time to enqueue the K steps
    if args.stream_sync:  # wait on the engine stream(s) first, then the device
        n_launch, win_ms = eng.timing_end()
        drain()
    else:  # the closing event recorded, one device-wide wait (covers every stream)
        eng.timing_stop()
    torch.cuda.synchronize()
    if _pg():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if not args.stream_sync:
        n_launch, win_ms = eng.timing_end()  # the window's events are complete: reads only
        drain()
    pairs_total_rank = rank_pairs(args.steps)  # pairs scored by this rank over the timed steps
    stats = torch.tensor([elapsed, pairs_total_rank], dtype=torch.float64, device="cuda")
    if _pg():
        t_max = stats[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        tot = stats[1:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed_max, pairs_all = float(t_max.item()), float(tot.item())
    else:
        elapsed_max, pairs_all = elapsed, pairs_total_rank

    ns = None
    if args.config == "c2" and not args.no_north_star:  # every rank (collectives inside)
        ns = north_star(args, world, rank, local)
    if rank == 0:
        value = pairs_all / elapsed_max
        cooc = args.model == "ibm" and eng.ibm_route == "cooc"
        ab_stage = (cooc_bytes(eng, ds, 4 if dense_out else 0, 10) if cooc
                    else algorithmic_bytes(ds, 4 if dense_out else 0, 10))
        if eng.fused:
            # one kernel per step: the window's mean is that kernel's mean launch
            # duration (plus the launch gaps, which the rocprof summary excludes)
            dom = "score"
            ab_dom = sum(ab_stage.values())
        else:
            dom = "steps"
            ab_dom = sum(ab_stage.values())
        # the launches of one step run back to back on the engine stream: the
        # window over K steps / K is the step's device time (= the fused
        # kernel's launch time at C2; all of a step's kernels otherwise)
        avg_us = win_ms / max(args.steps, 1) * 1e3
        launches_per_step = n_launch / max(args.steps, 1)
        achieved = ab_dom / (avg_us * 1e-6) / 1e9
        step_bytes = sum(ab_stage.values())
        traffic, traffic_src = args.traffic_bytes, "--traffic-bytes" if args.traffic_bytes else None
        pmc_file = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
        if traffic is None and os.path.exists(pmc_file) and world == 1 and args.inflight == 1:
            with open(pmc_file) as f:
                pmc = json.load(f)
            # counters of the same ibm route only (a wide-shape file without the key is two-hop)
            route = eng.ibm_route if (args.model == "ibm" and eng.shape == "wide") else None
            if route is None or (pmc.get("ibm_route") or "two_hop") == route:
                traffic = pmc.get("traffic_bytes_per_launch")
                traffic_src = (f"profiles/pmc_{args.config}.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                               f"of this command)")
        # quality companions on the last step's outputs (host-side, untimed)
        from musicrecommendation_amd import evaluation

        if args.shard == "users" and not bulk:
            songs, _sc, _k = eng.topk()
            map10 = evaluation.map_at_k(songs, ds, 10)
            ref_map = evaluation.threshold_map(eng.dense().astype(np.float64), ds) if dense_out else None
        else:
            s_, _k = scorer.topk()
            map10 = evaluation.map_at_k(s_, ds, 10)  # this rank's user block
            ref_map = None
        line = {
            "metric": "scored (test-user,song) pairs/sec, ItemBasedModel, 1/2/4/8 MI355X + mAP@10"
            if args.model == "ibm" else "scored (test-user,song) pairs/sec, UserBasedModel",
            "value": value,
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if bulk else "weak",
            # README's parallel-Scala number is quoted on C2's shape (500 / 10) only
            "vs_baseline": value / SCALA_PAR_PAIRS_PER_S if args.model == "ibm" and args.config == "c2" else None,
            "dtype": "int64",
            "data": "synthetic (seeded Zipf/lognormal Taste-Profile-shaped triplets, SURVEY.md §8d)",
            "config": {
                "workload": f"{args.config}: {'ItemBasedModel' if args.model == 'ibm' else 'UserBasedModel'} "
                            f"{n_tr} train / {n_te} test {'in total' if bulk else 'per GPU'} / "
                            f"{full.n_songs} songs, {'fp32 dense scores + ' if dense_out else ''}top-10, "
                            f"shard={args.shard}",
                "n_train": n_tr, "n_test": full.n_test, "n_songs": full.n_songs,
                "pairs_per_step": pairs_all / args.steps,
                "parallelism": (f"users{world}" if args.shard == "users" and not bulk
                                else f"songs{scorer.gs}xusers{scorer.gu}"),
                "inflight": args.inflight,
                "launch": (f"hip graph of {g_steps} steps x {args.steps // g_steps}" if use_graph
                           else "stream launches"),
                "host_submit_ms": t_submit * 1e3,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": ("k_cooc_build + k_cooc_light + k_score_wide<cooc> + k_topk_merge (per step)" if cooc else
                           {"fused": "k_score (fused: stages 1+2+3, one launch per step)",
                            "separate": "k_neighbours + k_score (per step)",
                            "wide": "k_neighbours + k_score_wide + k_topk_merge (per step)"}[eng.shape]),
                "byte_model": ("co-listening route (bench.cooc_bytes: index build + rows read per user)" if cooc
                               else "two-hop (bench.algorithmic_bytes, SURVEY.md §8d)"),
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                # measured fabric bytes over the same device time (traffic per launch ÷ avg_launch_us)
                "traffic_GBps": traffic / (avg_us * 1e-6) / 1e9 if traffic else None,
                # measured fetched + written bytes over the same device time, as a fraction of
                # the 8 TB/s peak: the fabric saturation (frac counts algorithmic bytes only)
                "traffic_frac": traffic / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS if traffic else None,
                "algorithmic_bytes_per_launch": ab_dom,
                "avg_launch_us": avg_us,
                "launches_per_step": launches_per_step,
                "timing": f"HIP events on the engine stream around the {args.steps} timed steps "
                          f"({n_launch} scoring launches; avg_launch_us = device time per step)",
            },
            "launch": {"shape": eng.shape, "block_songs": eng.block_songs, "n_tiles": eng.n_tiles,
                       "ibm_route": eng.ibm_route},
            "step_algorithmic_bytes": step_bytes,
            "step_GBps": step_bytes / (elapsed_max / args.steps) / 1e9,
            "mAP@10": map10,
            "ref_threshold_mAP": ref_map,
        }
        if args.config == "c1":  # config 1 names the reference's sequential Scala path
            line["vs_baseline"] = value / SCALA_C1_UBM_SEQ_PAIRS_PER_S if args.model == "ubm" else None
        if world == 1 and not args.no_cpu_baseline:
            if bulk or args.config == "c3":  # the literal loop nest is infeasible past C2
                line["cpu_baseline"] = cpu_baseline_twohop(ds, args.model, args.cpu_baseline_seconds)
            elif args.config == "c1":
                line["cpu_baseline"] = cpu_baseline_sequential(ds, args.model)
                line["cpu_baseline_par"] = cpu_baseline(ds, args.model, args.cpu_baseline_seconds)
            else:
                line["cpu_baseline"] = cpu_baseline(ds, args.model, args.cpu_baseline_seconds)
        else:
            line["cpu_baseline"] = None
        if world == 1 and not bulk and not args.no_e2e:
            line["end_to_end"] = end_to_end(ds, args.model)
        if world == 1 and bulk and not args.no_e2e and trip is not None:
            line["end_to_end"] = end_to_end_bulk(trip, args.model)
        if ns is not None:
            line["north_star"] = ns
        print(json.dumps(line), flush=True)
    for e in engines:
        e.close()
    if _pg():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
