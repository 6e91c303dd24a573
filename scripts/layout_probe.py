"""Per-rank device time of the multi-GPU layouts at C4, measured one rank at a
time on ONE GPU (the driver's 8-GPU node is not available to this build's
sessions). Rank r of a G_s x G_u layout scores user block r // G_s over song
shard r % G_s (sharding.ShardScorer / mr_group_*): the same Engine slice is
built here and its mr_run timed with HIP events on the engine stream (top-k
only, as bench.py --config c4). The slowest rank bounds a step; the exchange
(one all-gather of n_block x k x 12 B per block + k_topk_merge, ~10 us) is
not included.
  python scripts/layout_probe.py [model] [layouts, e.g. 1x1,8x1,4x2,2x4,1x8]"""
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
    model = sys.argv[1] if len(sys.argv) > 1 else "ibm"
    spec = sys.argv[2] if len(sys.argv) > 2 else "1x1,8x1,4x2,2x4,1x8"
    tiled = os.environ.get("MR_PROBE_UNTILED") is None  # shard boundaries at whole wide tiles (default)
    layouts = [tuple(int(x) for x in s.split("x")) for s in spec.split(",")]
    full = c4_dataset()
    base = None
    for gs, gu in layouts:
        t0 = time.time()
        tile = shard_tile(full.n_train, full.n_test // gu, n_songs=full.n_songs, n_shards=gs) if tiled else 0
        shards = song_shards(full, gs, tile)
        blocks = user_blocks(full.n_test, gu)
        ranks = []
        for r in range(gs * gu):
            (a, b), (lo, hi) = blocks[r // gs], shards[r % gs]
            ds = full if gu == 1 else full.subset_test_users(a, b)
            with Engine(ds, topk=10, dense=False, song_lo=lo, song_hi=hi,
                        ibm_route=os.environ.get("MR_PROBE_ROUTE", "auto")) as e:
                e.run(model)
                e.sync()
                e.timing_begin()
                e.run(model)
                _n, ms = e.timing_end()
                ranks.append({"rank": r, "users": [a, b], "songs": [lo, hi], "n_tiles": e.n_tiles,
                              "batch": e.batch, "ibm_route": e.ibm_route, "device_ms": ms})
        worst = max(x["device_ms"] for x in ranks)
        if (gs, gu) == (1, 1):
            base = worst
        out = {"layout": f"{gs}x{gu}", "model": model, "tiled_shards": tiled, "max_rank_ms": worst,
               "mean_rank_ms": sum(x["device_ms"] for x in ranks) / len(ranks),
               "speedup_vs_1x1": base / worst if base else None, "ranks": ranks, "wall_s": time.time() - t0}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
