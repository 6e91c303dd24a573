"""C4 wide-shape probe: one neighbour batch of the full Taste Profile shape.

Generates synth.config("c4") once per box (cached under $TMPDIR as .npz), then
runs the engine top-k only on the first N test users (default: one full
neighbour batch of the wide shape) — so a rocprofv3 --pmc pass sees one
k_neighbours + one k_score_wide + one k_topk_merge dispatch per run.
  python scripts/c4_probe.py [N_USERS] [model]      timing (+ JSON on stdout)
  MR_PROBE_CHUNK=C ...                              stage-1 chunk of C train users
  MR_PROBE_BS=B ...                                 song tiles of B songs
  MR_PROBE_BYTES=1 ...                              + the byte model per dispatch:
      algorithmic and the wide kernel's per-(neighbour, tile)
      index re-walk (nbr_v 4 B + nbr_q 8 B + toff pair 8 B, x n_tiles)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.dataset import Dataset  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

CACHE = os.path.join(os.environ.get("TMPDIR", "/tmp"), "mr_c4_triplets.npz")


def c4_dataset():
    if os.path.exists(CACHE):
        z = np.load(CACHE)
        return Dataset.from_triplets(z["tu"], z["ts"], z["eu"], z["es"], z["lu"], z["ls"])
    t = synth.config("c4")
    np.savez(CACHE, tu=t.train_u, ts=t.train_s, eu=t.test_u, es=t.test_s, lu=t.label_u, ls=t.label_s)
    return t.dataset()


def byte_model(ds, n_tiles, k=10):
    """Per dispatch, for the probe's users: algorithmic bytes of stage 1 / 2 / 3
    (bench.algorithmic_bytes, top-k only) and the wide kernel's index re-walk."""
    from bench import algorithmic_bytes

    ab = algorithmic_bytes(ds, 0, k)
    n_s = ds.n_songs
    tr_deg = np.diff(ds.tr_off)
    trs_ptr = np.zeros(n_s + 1, dtype=np.int64)
    np.cumsum(np.bincount(ds.tr_songs, minlength=n_s), out=trs_ptr[1:])
    order = np.argsort(ds.tr_songs, kind="stable")
    trs_users = np.repeat(np.arange(ds.n_train), tr_deg)[order]
    mark = np.zeros(ds.n_train, dtype=bool)
    nbrs = entries = 0
    for u in range(ds.n_test):
        T = ds.te_songs[ds.te_off[u]:ds.te_off[u + 1]]
        flat = np.concatenate([trs_users[trs_ptr[s]:trs_ptr[s + 1]] for s in T])
        mark[flat] = True
        nb = np.flatnonzero(mark)
        mark[flat] = False
        nbrs += nb.size
        entries += int(tr_deg[nb].sum())
    return {"algorithmic": ab, "neighbours": nbrs, "neighbour_song_entries": entries,
            "rewalk_index_bytes": nbrs * n_tiles * 20, "segment_song_bytes": entries * 2,
            "lds_atomics": entries}


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 704
    model = sys.argv[2] if len(sys.argv) > 2 else "ibm"
    t0 = time.time()
    full = c4_dataset()
    t1 = time.time()
    ds = full.subset_test_users(0, n)
    with Engine(ds, topk=10, dense=False, stage1_chunk=int(os.environ.get("MR_PROBE_CHUNK", "0")),
                block_songs=int(os.environ.get("MR_PROBE_BS", "0"))) as e:
        t2 = time.time()
        e.run(model)
        e.sync()
        e.timing_begin()
        e.run(model)
        launches, ms = e.timing_end()
        out = {"users": n, "batch": e.batch, "n_tiles": e.n_tiles, "block_songs": e.block_songs,
               "n_chunks": e.n_chunks, "device_ms": ms, "dataset_s": t1 - t0, "load_s": t2 - t1}
    if os.environ.get("MR_PROBE_BYTES"):
        out["bytes"] = byte_model(ds, out["n_tiles"])
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
