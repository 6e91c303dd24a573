"""Census of C4's co-listening index rows: rows =
distinct test-visible songs with train listeners, classified light / heavy
as mr_load does (entry bound min(Σ_{v ∈ L_tr(s2)} |S(v)|, n_s) within 80 % of
32,768 hash slots and ≤ 4,095 listeners), and per class the listeners, the
entries the build reads, how many test users read each row (te_cnt) and the
(user, listener) pairs a listener-list scoring would walk.
  python scripts/light_rows_census.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from c4_probe import c4_dataset  # noqa: E402

t0 = time.time()
ds = c4_dataset()
print("dataset", round(time.time() - t0, 1), "s", flush=True)
n_s, n_tr = ds.n_songs, ds.n_train
deg = np.diff(ds.tr_off).astype(np.int64)
c_tr = np.bincount(ds.tr_songs, minlength=n_s).astype(np.int64)
owner = np.repeat(np.arange(n_tr), deg)
sdeg = np.bincount(ds.tr_songs, weights=deg[owner], minlength=n_s).astype(np.int64)
te_cnt = np.bincount(ds.te_songs, minlength=n_s)
rows = np.nonzero((te_cnt > 0) & (c_tr > 0))[0]
bound = np.minimum(sdeg[rows], n_s)
light = (bound * 100 <= 32768 * 80) & (c_tr[rows] <= 4095)
print("rows", rows.size, "light", int(light.sum()), "heavy", int((~light).sum()))
for name, R in (("light", rows[light]), ("heavy", rows[~light])):
    print(name, "listeners", int(c_tr[R].sum()), "entries", int(sdeg[R].sum()), "te_cnt mean",
          round(float(te_cnt[R].mean()), 4), "te_cnt==1", round(float((te_cnt[R] == 1).mean()), 4),
          "listeners median", float(np.median(c_tr[R])), "user-listener pairs", int((te_cnt[R] * c_tr[R]).sum()))
L = rows[light]
for thr in (1, 2, 3):
    m = te_cnt[L] <= thr
    print(f"light rows te_cnt<={thr}: {int(m.sum())} rows, listeners {int(c_tr[L][m].sum())}, entries "
          f"{int(sdeg[L][m].sum())}, user-listener pairs {int((te_cnt[L][m] * c_tr[L][m]).sum())}")
