"""Count distribution of the co-listening index as the scoring reads it (C4 1x1).

The scoring kernel reads, per test user u and tile, the segments of u's index
rows s2: dense segments (a count byte per song, saturated at 255 + excess
entries) and sparse ones (4-B entries (song << 17) | C). Each (row, tile)
segment is read once per test user holding s2, so this script weights every
row by te_cnt(s2) (its test users) and reports, over the bytes the scoring
consumes: the count histogram of dense songs and of sparse entries, and the
bytes of alternative encodings (a nibble per dense song saturated at 15 + 4-B
excess entries; sparse entries with C = 1 (or C <= 2) as 2-B song ids).

Rows: the heaviest rows by consumption exactly, a uniform sample of the rest
(weight 1 / rate). Dense rule as mr_load's: non-zeros * 3 >= the tile's songs.

usage: python scripts/count_hist.py [--exact N] [--rate R] [--out FILE]
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from musicrecommendation_amd import synth  # noqa: E402

BS, DENSE_DIV = 19456, 3


def arg(name, default, cast):
    return cast(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    n_exact, rate, out = arg("--exact", 3000, int), arg("--rate", 0.05, float), arg("--out", None, str)
    t0 = time.time()
    ds = synth.config("c4").dataset()
    n_tr, n_s = ds.n_train, ds.n_songs
    deg = np.diff(ds.tr_off)
    A = sp.csr_matrix((np.ones(ds.tr_songs.size, np.int32), ds.tr_songs.astype(np.int64), ds.tr_off),
                      shape=(n_tr, n_s))
    AT = A.T.tocsr()
    c_tr = np.diff(AT.indptr)
    te_cnt = np.bincount(ds.te_songs.astype(np.int64), minlength=n_s)
    rows = np.nonzero((te_cnt > 0) & (c_tr > 0))[0]
    # consumption proxy: test users x listeners' entries (bound of the row's entries)
    bound = np.add.reduceat(deg[AT.indices], AT.indptr[:-1].clip(max=AT.indices.size - 1))[rows]
    cons = te_cnt[rows] * np.minimum(bound, n_s)
    order = np.argsort(-cons, kind="stable")
    exact = rows[order[:n_exact]]
    rest = rows[order[n_exact:]]
    rng = np.random.default_rng(1)
    samp = rest[rng.random(rest.size) < rate]
    n_tiles = (n_s + BS - 1) // BS
    H = 1 << 17
    dense_hist = np.zeros(H, np.float64)   # count -> weighted dense songs
    sparse_hist = np.zeros(H, np.float64)  # count -> weighted sparse entries
    seg = {"dense_segments": 0.0, "sparse_segments": 0.0}
    for group, w in ((exact, 1.0), (samp, 1.0 / rate)):
        for s2 in group:
            lst = AT.indices[AT.indptr[s2]:AT.indptr[s2 + 1]]
            cnt = np.bincount(A[lst].indices, minlength=n_s)
            wt = w * te_cnt[s2]
            for t in range(n_tiles):
                c = cnt[t * BS:min(n_s, (t + 1) * BS)]
                nz = c[c > 0]
                if nz.size == 0:
                    continue
                if nz.size * DENSE_DIV >= c.size:
                    dense_hist += wt * np.bincount(np.minimum(c, H - 1), minlength=H)
                    seg["dense_segments"] += wt
                else:
                    sparse_hist += wt * np.bincount(np.minimum(nz, H - 1), minlength=H)
                    seg["sparse_segments"] += wt
    d_songs, s_ent = dense_hist.sum(), sparse_hist.sum()

    def frac(h, lo, hi):
        return float(h[lo:hi + 1].sum() / max(h.sum(), 1))

    cur_exc = float((dense_hist[256:]).sum())  # dense songs with an excess entry now
    res = {
        "rows": int(rows.size), "exact_rows": int(exact.size), "sampled_rows": int(samp.size), "rate": rate,
        "consumed_dense_songs": d_songs, "consumed_sparse_entries": s_ent, **seg,
        "dense_count_fractions": {"0": frac(dense_hist, 0, 0), "1": frac(dense_hist, 1, 1),
                                  "2-3": frac(dense_hist, 2, 3), "4-7": frac(dense_hist, 4, 7),
                                  "8-15": frac(dense_hist, 8, 15), "16-255": frac(dense_hist, 16, 255),
                                  ">255": frac(dense_hist, 256, H)},
        "sparse_count_fractions": {"1": frac(sparse_hist, 1, 1), "2": frac(sparse_hist, 2, 2),
                                   "3": frac(sparse_hist, 3, 3), "4-15": frac(sparse_hist, 4, 15),
                                   ">15": frac(sparse_hist, 16, H)},
    }
    GB = 1e9
    now = d_songs + 4 * (s_ent + cur_exc)
    nib = 0.5 * d_songs + 4 * (s_ent + float(dense_hist[16:].sum()))
    ones = d_songs + 4 * cur_exc + 2 * float(sparse_hist[1]) + 4 * float(sparse_hist[2:].sum())
    two = d_songs + 4 * cur_exc + 2 * float(sparse_hist[1:3].sum()) + 4 * float(sparse_hist[3:].sum())
    both = 0.5 * d_songs + 4 * float(dense_hist[16:].sum()) + 2 * float(sparse_hist[1:3].sum()) \
        + 4 * float(sparse_hist[3:].sum())
    res["consumed_GB"] = {"now": now / GB, "dense_nibbles": nib / GB, "sparse_ones_u16": ones / GB,
                          "sparse_le2_u16": two / GB, "nibbles_and_le2_u16": both / GB}
    res["seconds"] = time.time() - t0
    print(json.dumps(res, indent=1))
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
