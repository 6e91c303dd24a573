"""Phase times of the co-listening index build in the diagnostic build
libmr_engine_stamps.so (s_memrealtime, 100 MHz): every light row (k_cooc_light /
k_cooc_light_wave: start, table zeroed, listeners walked, tile counts, end) and
every heavy-row workgroup (k_cooc_group: start, first group walked, first
group's tiles emitted, end), for C4 or one song shard of it.
Usage: [SHARD=g/G] python scripts/cooc_build_stamps.py"""
import os
import sys

os.environ.setdefault("MR_ENGINE_LIB", "stamps")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import numpy as np  # noqa: E402

from c4_probe import c4_dataset  # noqa: E402
from musicrecommendation_amd.engine import Engine  # noqa: E402
from musicrecommendation_amd.sharding import shard_tile, song_shards  # noqa: E402

ds = c4_dataset()
lo, hi = 0, 0
if os.environ.get("SHARD"):
    g, G = (int(x) for x in os.environ["SHARD"].split("/"))
    lo, hi = song_shards(ds, G, shard_tile(ds.n_train, ds.n_test, n_songs=ds.n_songs, n_shards=G))[g]
with Engine(ds, topk=10, dense=False, song_lo=lo, song_hi=hi, ibm_route="cooc") as e:
    for _ in range(2):
        e.run("ibm")
        e.sync()
    cb = e.cooc_bytes()
    nt = e.n_tiles
    users = max(e.batch, min(ds.n_test, 65528)) + 8
    boff = nt * users * 32
    build_wgs = cb["heavy_rows"] * nt + 64 * nt
    loff = boff + build_wgs * 8
    total = loff + cb["light_rows"] * 8
    buf = np.zeros(total, dtype=np.int64)
    assert e._L.mr_debug_stamps(e._h, buf.ctypes.data, buf.size) == 0
tick_us = 0.01
L = buf[loff:].reshape(-1, 8)
print(f"shard [{lo},{hi}) tiles {nt}: light rows {len(L)}, heavy rows {cb['heavy_rows']}, "
      f"groups {cb['n_groups']} x {cb['group_tiles']} tiles")
# a row is decoded only when every phase slot was written and the slots ascend
# (the diagnostic kernels write slots 0-4 in order; a 0 = a phase never stamped)
lok = (L[:, :5] > 0).all(axis=1) & (np.diff(L[:, :5], axis=1) >= 0).all(axis=1)
if (~lok & (L[:, 0] > 0)).any():
    print(f" light rows with incomplete stamps (dropped): {int((~lok & (L[:, 0] > 0)).sum())}")
t_all0 = L[:, 0][L[:, 0] > 0].min() if (L[:, 0] > 0).any() else 0
for (S, NT) in sorted({(int(a), int(b)) for a, b in L[lok][:, 6:8] if a > 0}, reverse=True):
    m = (L[:, 6] == S) & (L[:, 7] == NT) & lok
    x = L[m].astype(np.float64)
    ph = {"zero": x[:, 1] - x[:, 0], "walk": x[:, 2] - x[:, 1], "count": x[:, 3] - x[:, 2],
          "emit": x[:, 4] - x[:, 3]}
    dur = x[:, 4] - x[:, 0]
    span = (x[:, 4].max() - x[:, 0].min()) * tick_us
    n = x[:, 5]
    print(f" tier S={S:5d} NT={NT:4d}: rows {m.sum():6d} listeners {int(n.sum()):9d} span {span / 1e3:7.2f} ms "
          f"(start {(x[:, 0].min() - t_all0) * tick_us / 1e3:6.2f} ms) row med {np.median(dur) * tick_us:8.1f} us")
    for k, v in ph.items():
        print(f"    {k:6s} med {np.median(v) * tick_us:8.1f} us  p90 {np.percentile(v, 90) * tick_us:8.1f}  "
              f"share {v.sum() / dur.sum():.3f}")
    w = ph["walk"] * tick_us
    print(f"    walk per listener med {np.median(w / np.maximum(n, 1)) * 1e3:8.1f} ns")
B = buf[boff:loff].reshape(-1, 8)
B = B[B[:, 0] > 0]
# complete workgroups only: slots 0 <= 1 <= 3 <= 2 <= 4 all written (k_cooc_build
# writes slot 3 = slot 2: no pass split)
bok = (B[:, :5] > 0).all(axis=1) & (B[:, 1] >= B[:, 0]) & (B[:, 3] >= B[:, 1]) & (B[:, 2] >= B[:, 3]) & \
    (B[:, 4] >= B[:, 2])
if (~bok).any():
    print(f" heavy WGs with incomplete stamps (dropped): {int((~bok).sum())}")
B = B[bok].astype(np.float64)
if len(B):
    dur = (B[:, 4] - B[:, 0]) * tick_us
    print(f" heavy WGs {len(B)} (big {int(B[:, 5].sum())}), span {(B[:, 4].max() - B[:, 0].min()) * tick_us / 1e3:.2f} ms, "
          f"sum(WG time)/256 {dur.sum() / 256 / 1e3:.2f} ms")
    b32 = B[:, 7] == -1  # k_cooc_build: the u32 rows, one workgroup per (row, tile)
    g = ~b32             # k_cooc_group (slot 7: its group count, 1 for big rows)
    for kind, sel in (("pipelined rows", g & (B[:, 5] == 0)), ("big rows (row, group)", g & (B[:, 5] == 1)),
                      ("u32 rows (row, tile), k_cooc_build", b32)):
        if not sel.any():
            continue
        print(f"   {kind}: WGs {sel.sum()} med {np.median(dur[sel]):8.1f} us, share {dur[sel].sum() / dur.sum():.3f}")
        for name, a, b in (("first walk", 0, 1), ("first emit", 1, 2), (" pass A", 1, 3), (" pass B", 3, 2),
                           ("rest", 2, 4)):
            v = (B[sel, b] - B[sel, a]) * tick_us
            print(f"    {name:10s} med {np.median(v):8.1f} us p90 {np.percentile(v, 90):8.1f} "
                  f"share {v.sum() / dur[sel].sum():.3f}")
    n = B[:, 6]
    for lo_, hi_ in ((0, 4096), (4096, 16384), (16384, 1 << 30)):
        m = (n >= lo_) & (n < hi_)
        if m.any():
            print(f"    listeners [{lo_},{hi_}): WGs {m.sum():6d} med {np.median(dur[m]):9.1f} us, walk per listener "
                  f"{np.median((B[m, 1] - B[m, 0]) * tick_us / n[m]) * 1e3:7.1f} ns, share {dur[m].sum() / dur.sum():.3f}")
