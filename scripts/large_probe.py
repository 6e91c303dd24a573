"""Probe of the large-train-set path (config 4 shape): build a bulk synthetic
dataset, time top-k-only runs of the engine, check sampled users bit for bit
against the fixed-point oracle. Usage: python scripts/large_probe.py N_TRAIN N_TEST [model] [block]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402
from oracle import native  # noqa: E402

n_tr, n_te = int(sys.argv[1]), int(sys.argv[2])
model = sys.argv[3] if len(sys.argv) > 3 else "ibm"
block = int(sys.argv[4]) if len(sys.argv) > 4 else 0
dense = os.environ.get("DENSE", "0") == "1"
t = time.time()
ds = synth.generate_bulk(n_tr, n_te, 4).dataset()
print(f"dataset {n_tr}/{n_te}: {ds.n_songs} songs, {int(ds.tr_off[-1])} train rows, {time.time() - t:.1f} s", flush=True)
t = time.time()
with Engine(ds, topk=10, dense=dense, block_songs=block) as e:
    print(f"load {time.time() - t:.1f} s shape={e.shape} bs={e.block_songs} tiles={e.n_tiles}", flush=True)
    e.run(model)
    e.sync()
    for it in range(3):
        t = time.perf_counter()
        e.timing_begin()
        e.run(model)
        n, ms = e.timing_end()
        dt = time.perf_counter() - t
        print(f"run {it}: {ms:.2f} ms device, {dt * 1e3:.2f} ms wall, {ds.n_pairs() / (ms * 1e-3):.3e} pairs/s", flush=True)
    songs, _, keys = e.topk()
users = [0, n_te // 2, n_te - 1]
for u in users:
    _, ts, tk = native.fp_model(ds, model, user_lo=u, user_hi=u + 1, k=10, dense=False)
    ok = np.array_equal(songs[u:u + 1], ts) and np.array_equal(keys[u:u + 1], tk)
    print(f"user {u}: top-k exact {ok}", flush=True)
    if not ok:
        sys.exit(1)
