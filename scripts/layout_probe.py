"""Per-rank device time of the multi-GPU layouts at C4, measured one rank at a
time on ONE GPU (the driver's 8-GPU node is not available to this build's
sessions). Rank r of a G_s x G_u layout scores user block r // G_s over song
shard r % G_s (sharding.ShardScorer / mr_group_*): the same Engine slice is
built here and its mr_run timed with HIP events on the engine stream (top-k
only, as bench.py --config c4). The slowest rank bounds a step; the exchange
(one all-gather of n_block x k x 12 B per block + k_topk_merge, ~10 us) is
not included.
  python scripts/layout_probe.py [model] [layouts, e.g. 1x1,8x1,4x2,2x4,1x8]
  MR_PROBE_BS=B   song tiles of B songs (block_songs) instead of the engine's choice
  MR_PROBE_CONFIG=c5 MR_PROBE_DENSE=1 python scripts/layout_probe.py ubm,ibm 1x1,8x1,2x4
                  C5's two dense models per rank (the ensemble's scoring passes)
  MR_PROBE_REPS=R timed runs per rank (the minimum is reported; default 1)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch  # noqa: E402,F401

from c4_probe import c4_dataset  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402
from musicrecommendation_amd.sharding import shard_tile, song_shards, user_blocks  # noqa: E402


def main():
    models = (sys.argv[1] if len(sys.argv) > 1 else "ibm").split(",")
    spec = sys.argv[2] if len(sys.argv) > 2 else "1x1,8x1,4x2,2x4,1x8"
    tiled = os.environ.get("MR_PROBE_UNTILED") is None  # shard boundaries at whole wide tiles (default)
    layouts = [tuple(int(x) for x in s.split("x")) for s in spec.split(",")]
    cfg = os.environ.get("MR_PROBE_CONFIG", "c4")
    dense = os.environ.get("MR_PROBE_DENSE") == "1"  # C5: the dense f32 models of the ensemble
    if cfg == "c4":
        full = c4_dataset()
    else:
        from musicrecommendation_amd import synth

        full = synth.config(cfg).dataset()
    base = None
    bs = int(os.environ.get("MR_PROBE_BS", "0"))
    reps = int(os.environ.get("MR_PROBE_REPS", "1"))
    for gs, gu in layouts:
        t0 = time.time()
        tile = shard_tile(full.n_train, full.n_test // gu, n_songs=full.n_songs, n_shards=gs,
                          block_songs=bs) if tiled else 0
        shards = song_shards(full, gs, tile)
        blocks = user_blocks(full.n_test, gu)
        ranks = []
        for r in range(gs * gu):
            (a, b), (lo, hi) = blocks[r // gs], shards[r % gs]
            ds = full if gu == 1 else full.subset_test_users(a, b)
            with Engine(ds, topk=10, dense=dense, song_lo=lo, song_hi=hi, block_songs=bs,
                        ibm_route=os.environ.get("MR_PROBE_ROUTE", "auto")) as e:
                per_model = {}
                for model in models:
                    e.run(model)
                    e.sync()
                    times = []
                    for _ in range(reps):
                        e.timing_begin()
                        e.run(model)
                        _n, ms = e.timing_end()
                        times.append(ms)
                    per_model[model] = min(times)
                ranks.append({"rank": r, "users": [a, b], "songs": [lo, hi], "n_tiles": e.n_tiles,
                              "block_songs": e.block_songs, "batch": e.batch, "ibm_route": e.ibm_route,
                              "device_ms": sum(per_model.values()), "device_ms_per_model": per_model})
        worst = max(x["device_ms"] for x in ranks)
        if (gs, gu) == (1, 1):
            base = worst
        out = {"layout": f"{gs}x{gu}", "config": cfg, "models": models, "dense": dense, "tiled_shards": tiled,
               "max_rank_ms": worst,
               "mean_rank_ms": sum(x["device_ms"] for x in ranks) / len(ranks),
               "speedup_vs_1x1": base / worst if base else None, "ranks": ranks, "wall_s": time.time() - t0}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
