"""Per-workgroup phase timestamps of the large-train-set path (diagnostic
build libmr_engine_stamps.so). Usage: python scripts/large_stamps.py N_TRAIN N_TEST [model] [block]"""
import os
import sys

os.environ.setdefault("MR_ENGINE_LIB", "stamps")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from musicrecommendation_amd import synth  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402

n_tr, n_te = int(sys.argv[1]), int(sys.argv[2])
model = sys.argv[3] if len(sys.argv) > 3 else "ibm"
block = int(sys.argv[4]) if len(sys.argv) > 4 else 0
if os.environ.get("CONFIG"):  # e.g. CONFIG=c2 STAGE1=wide: a bench config instead of bulk synthetic
    ds = synth.config(os.environ["CONFIG"]).dataset()
    n_tr, n_te = ds.n_train, ds.n_test
else:
    ds = synth.generate_bulk(n_tr, n_te, 4).dataset()
lo, hi = 0, 0
if os.environ.get("SHARD"):  # SHARD=g/G: song shard g of G (sharding.song_shards at the shard tile)
    from musicrecommendation_amd.sharding import shard_tile, song_shards

    g, G = (int(x) for x in os.environ["SHARD"].split("/"))
    tile = shard_tile(ds.n_train, ds.n_test, n_songs=ds.n_songs, n_shards=G, block_songs=block)
    lo, hi = song_shards(ds, G, tile)[g]
with Engine(ds, topk=10, dense=bool(os.environ.get("DENSE")), block_songs=block, song_lo=lo, song_hi=hi,
            stage1=os.environ.get("STAGE1", "auto")) as e:
    e.run(model)
    e.sync()
    e.run(model)
    e.sync()
    gy = (n_te + 7) // 8 * 8
    n = e.n_tiles * gy
    buf = np.zeros(n * 32, dtype=np.int64)
    rc = e._L.mr_debug_stamps(e._h, buf.ctypes.data, buf.size)
    assert rc == 0
    tiles = e.n_tiles
full = buf.reshape(n, 32)
lin = np.arange(n)
slot = lin >> 3
bu = (slot // tiles) * 8 + (lin & 7)
live = (bu < n_te) & (full[:, 0] != 0)
rt = full[:, :16].astype(np.float64) * 10.0 / 1e3  # us
rt, bu = rt[live], bu[live]
t0 = rt[:, 0].min()
end = rt[:, 5]
span = end.max() - t0
dur = end - rt[:, 0]
print(f"{n_tr}/{n_te} {model}: tiles={tiles} WGs={live.sum()} kernel span {span / 1e3:.2f} ms; "
      f"sum(WG time)/256 = {dur.sum() / 256 / 1e3:.2f} ms")
for name, a, b in (("prefix", 0, 1), ("stage2", 1, 2), (" cooc descr", 1, 12), (" cooc dense", 12, 13),
                   (" cooc sparse", 13, 14), ("epilogue", 2, 3), ("tile-topk", 3, 4), ("handoff", 4, 5),
                   (" topk scan", 3, 6), (" topk wave", 6, 7), (" topk barrier", 7, 8), (" topk merge", 8, 4),
                   (" thr pass1", 3, 9), (" thr rank", 9, 10), (" thr pass2", 10, 11), (" thr select", 11, 4)):
    d = rt[:, b] - rt[:, a]
    print(f"  {name:10s} us med {np.median(d):9.1f} p90 {np.percentile(d, 90):9.1f} max {d.max():9.1f} "
          f"sum share {d.sum() / dur.sum():.3f}")
# concurrency over time
ts = np.linspace(t0, end.max(), 20)
conc = [int(((rt[:, 0] <= t) & (end > t)).sum()) for t in ts]
print("concurrent WGs over time:", conc)
# stage-2 time per user vs its neighbour count
ctr = np.bincount(ds.tr_songs, minlength=ds.n_songs)
trs_off = np.zeros(ds.n_songs + 1, np.int64)
np.cumsum(ctr, out=trs_off[1:])
order = np.argsort(ds.tr_songs, kind="stable")
trs_users = np.repeat(np.arange(ds.n_train), np.diff(ds.tr_off))[order]
deg = np.diff(ds.tr_off)
rows = []
for u in range(0, n_te, max(1, n_te // 16)):
    T = ds.te_songs[ds.te_off[u]:ds.te_off[u + 1]]
    nb = np.unique(np.concatenate([trs_users[trs_off[s]:trs_off[s + 1]] for s in T]))
    s2 = rt[bu == u, 2] - rt[bu == u, 1]
    rows.append((u, nb.size, int(deg[nb].sum()), float(np.median(s2)), float(s2.max())))
for u, nn, ee, med, mx in rows:
    print(f"  user {u:5d} |N| {nn:7d} E {ee:9d} stage2 med {med:8.1f} us max {mx:8.1f} us"
          f"  -> {nn / med:.1f} visits/us, {ee / tiles / med:.1f} entries/us per WG")
