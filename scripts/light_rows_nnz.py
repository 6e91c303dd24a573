"""Light index rows of C4: their non-zeros (the union
of their listeners' songs) against the entry bound mr_load sizes their hash
tables by (Σ of the listeners' songs), on 300 sampled rows per table tier,
and the tiers the exact non-zeros would give (80 % load).
  python scripts/light_rows_nnz.py"""
import sys, time, numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c4_probe import c4_dataset
ds = c4_dataset()
n_s, n_tr = ds.n_songs, ds.n_train
deg = np.diff(ds.tr_off).astype(np.int64)
c_tr = np.bincount(ds.tr_songs, minlength=n_s).astype(np.int64)
owner = np.repeat(np.arange(n_tr), deg)
sdeg = np.bincount(ds.tr_songs, weights=deg[owner], minlength=n_s).astype(np.int64)
te_cnt = np.bincount(ds.te_songs, minlength=n_s)
rows = np.nonzero((te_cnt > 0) & (c_tr > 0))[0]
bound = np.minimum(sdeg[rows], n_s)
light = (bound * 100 <= 32768 * 80) & (c_tr[rows] <= 4095)
# transpose: song -> listeners
order = np.argsort(ds.tr_songs, kind='stable')
lst = owner[order]
soff = np.concatenate([[0], np.cumsum(c_tr)])
rng = np.random.default_rng(0)
def slots_for(b):
    s = 1024
    while s * 80 < b * 100: s <<= 1
    return s
L = rows[light]; B = bound[light]
tiers = np.array([slots_for(b) for b in B])
for S in (32768, 16384, 8192, 4096, 2048, 1024):
    idx = np.nonzero(tiers == S)[0]
    if idx.size == 0: continue
    samp = rng.choice(idx, size=min(300, idx.size), replace=False)
    ratios = []; newt = []
    for i in samp:
        s2 = L[i]
        vs = lst[soff[s2]:soff[s2+1]]
        songs = np.concatenate([ds.tr_songs[ds.tr_off[v]:ds.tr_off[v+1]] for v in vs])
        nnz = np.unique(songs).size
        ratios.append(nnz / B[i]); newt.append(slots_for(nnz))
    newt = np.array(newt)
    print(f"tier {S:5d}: rows {idx.size:6d} nnz/bound mean {np.mean(ratios):.3f} median {np.median(ratios):.3f}; "
          f"exact-nnz tiers: " + ", ".join(f"{t}:{(newt==t).mean():.2f}" for t in sorted(set(newt), reverse=True)), flush=True)
