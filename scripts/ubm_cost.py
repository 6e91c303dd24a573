"""Cost inputs of a song-factorised UserBasedModel route.

The ubm score factors through songs once its fixed-point weight is
o_v · rint(2^F / sqrt|S(v)|) (1/sqrt|T(u)| in the epilogue):
rank_u(u, s) = (2^-F / sqrt|T(u)|) Σ_{s2 ∈ T(u)} D[s2][s],
D[s2][s] = Σ_{v ∈ L_tr(s2) ∩ L_tr(s)} rint(2^F / sqrt|S(v)|) — the
co-listening index with weighted entries. D has the sparsity of the ibm
index C, so the ibm route's own counts of a config price it. This probe runs
the config's ibm model on the co-listening route and its ubm model on the
two-hop route (device time per run, median of reps) and prints the ibm
index's encoding counts (mr_cooc_bytes) as one JSON line.

usage: python scripts/ubm_cost.py [c5|c4] [reps]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402


def timed_runs(e, model, reps):
    out = []
    for _ in range(reps):
        e.sync()
        t0 = time.perf_counter()
        e.run(model)
        e.sync()
        out.append((time.perf_counter() - t0) * 1e3)
    out.sort()
    return out[len(out) // 2]


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    t0 = time.perf_counter()
    ds = synth.config(cfg).dataset()
    gen_s = time.perf_counter() - t0
    dense = cfg == "c5"
    res = {"config": cfg, "n_train": ds.n_train, "n_test": ds.n_test, "n_songs": ds.n_songs, "gen_s": gen_s}
    with Engine(ds, topk=10, dense=dense, out_dtype="f32", ibm_route="cooc") as e:
        res["block_songs"], res["n_tiles"] = e.block_songs, e.n_tiles
        e.run("ibm")
        e.sync()
        res["ibm_cooc_ms"] = timed_runs(e, "ibm", reps)
        res["cooc_bytes"] = e.cooc_bytes()
        res["cooc_rows"] = e.cooc_rows
        res["ubm_twohop_ms"] = timed_runs(e, "ubm", reps)
    print(json.dumps(res), flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
