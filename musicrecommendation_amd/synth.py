"""Seeded synthetic Taste-Profile-shaped triplets.

The real subsets (train_N_M.txt ...) are git-ignored in the reference and the
48M-row Echo Nest Taste Profile is not in this image, so every config runs on
synthetic data built to the split rule of the reference's data-prep notebook
(dataExtraction.ipynb):
  * song popularity Zipf(alpha) over 384,546 song ids (NB:126), randomly
    permuted onto ids;
  * history length max(10, round(lognormal(3.51, 0.86))) per user (fitted to
    NB cell 10: min 10, median 29, mean 53.2);
  * each user draws distinct songs; playcount 1 (ignored, MR:35);
  * train = first n_train users, test = next n_test (NB:149, NB:301);
  * each test user: first ceil(n/2) rows visible, the rest are labels (NB:571-573).
``alpha=None`` bisects alpha so that the number of distinct songs lands within
±5 % of ``target_songs`` (the README's song count for the named config).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .dataset import Dataset

N_SONG_UNIVERSE = 384_546  # distinct songs in the Taste Profile (NB:126)

# Named configs of BASELINE.json (n_train, n_test, seed, target distinct songs).
CONFIGS = {
    "c1": (100, 10, 1, 4798),      # README.md:72 (train_100_10)
    "c2": (500, 10, 2, 16785),     # README.md:96 (train_500_10)
    "c3": (10_000, 1_000, 3, None),
    "tiny": (20, 5, 7, None),
    "small": (60, 8, 11, None),
}
# alpha found by calibrate_alpha for the configs with a song-count target
# (cached so every run uses the same value; re-derive with calibrate_alpha).
ALPHA = {"c1": 0.7, "c2": 0.8625}


@dataclass
class Triplets:
    train_u: np.ndarray
    train_s: np.ndarray
    test_u: np.ndarray
    test_s: np.ndarray
    label_u: np.ndarray
    label_s: np.ndarray
    alpha: float

    def dataset(self) -> Dataset:
        return Dataset.from_triplets(self.train_u, self.train_s, self.test_u, self.test_s,
                                     self.label_u, self.label_s)

    def n_songs(self) -> int:
        return int(np.unique(np.concatenate([self.train_s, self.test_s])).size)

    def write_tsv(self, train_path: str, test_path: str, labels_path: str) -> int:
        """The three reference-format files (``user\tsong\t1`` lines in row
        order, names as dataset.user_name / song_name), written with numpy in
        blocks of rows: the full-scale files (48M lines, ~3 GB) in seconds.
        Returns the bytes written."""
        total = 0
        for path, u, s in ((train_path, self.train_u, self.train_s), (test_path, self.test_u, self.test_s),
                           (labels_path, self.label_u, self.label_s)):
            total += _write_triplet_file(path, u, s)
        return total


def _hex_names(keys: np.ndarray, prefix: bytes, width: int, upper: bool) -> np.ndarray:
    """Rows of fixed-width names prefix + hex(key) (dataset.user_name: 40 lower-case
    hex digits; song_name: "SO" + 16 upper-case), one uint8 row per key."""
    digits = np.frombuffer(b"0123456789ABCDEF" if upper else b"0123456789abcdef", dtype=np.uint8)
    out = np.empty((keys.size, len(prefix) + width), dtype=np.uint8)
    if prefix:
        out[:, :len(prefix)] = np.frombuffer(prefix, dtype=np.uint8)
    k = keys.astype(np.uint64)
    for i in range(width):
        out[:, len(prefix) + width - 1 - i] = digits[((k >> np.uint64(4 * i)) & np.uint64(15)).astype(np.intp)]
    return out


def _write_triplet_file(path: str, u: np.ndarray, s: np.ndarray, block: int = 1 << 22) -> int:
    uk, ui = np.unique(u, return_inverse=True)
    sk, si = np.unique(s, return_inverse=True)
    un = _hex_names(uk, b"", 40, False)
    sn = _hex_names(sk, b"SO", 16, True)
    wu, ws = un.shape[1], sn.shape[1]
    line = wu + ws + 4  # user \t song \t 1 \n
    with open(path, "wb") as f:
        for a in range(0, u.size, block):
            b = min(u.size, a + block)
            rows = np.empty((b - a, line), dtype=np.uint8)
            rows[:, :wu] = un[ui[a:b]]
            rows[:, wu] = 9
            rows[:, wu + 1:wu + 1 + ws] = sn[si[a:b]]
            rows[:, wu + 1 + ws:] = np.frombuffer(b"\t1\n", dtype=np.uint8)
            rows.tofile(f)
    return int(u.size) * line


def _user_songs(rng: np.random.Generator, cdf: np.ndarray, perm: np.ndarray) -> np.ndarray:
    """One user's history: length max(10, round(lognormal(3.51, 0.86))), distinct
    songs drawn by popularity (oversample with replacement, keep first draws)."""
    n_universe = cdf.size
    n = int(min(n_universe, max(10, round(float(rng.lognormal(3.51, 0.86))))))
    have = np.zeros(0, dtype=np.int64)
    for _ in range(64):
        ranks = np.searchsorted(cdf, rng.random(2 * n + 8), side="right")
        cat = np.concatenate([have, perm[np.minimum(ranks, n_universe - 1)]])
        _, first = np.unique(cat, return_index=True)
        first.sort()
        have = cat[first][:n]
        if have.size == n:
            return have
    raise RuntimeError("synthetic draw did not converge")


def _popularity(seed: int, alpha: float, n_universe: int):
    perm = np.random.default_rng([seed, 0]).permutation(n_universe).astype(np.int64)
    w = np.arange(1, n_universe + 1, dtype=np.float64) ** (-alpha)
    cdf = np.cumsum(w)
    cdf /= cdf[-1]
    return cdf, perm


def generate(n_train: int, n_test: int, seed: int, alpha: Optional[float] = None,
             target_songs: Optional[int] = None, n_universe: int = N_SONG_UNIVERSE,
             test_offset: int = 0) -> Triplets:
    """Train user i draws from stream (seed, 1, i), test user j from (seed, 2, j):
    datasets are prefix-consistent in n_train and n_test (the first 10 test
    users of a 500/40 dataset are those of 500/10)."""
    if alpha is None and target_songs is not None:
        alpha = calibrate_alpha(n_train, n_test, seed, target_songs, n_universe)
    if alpha is None:
        alpha = 0.87
    cdf, perm = _popularity(seed, alpha, n_universe)
    tr_u, tr_s = [], []
    for i in range(n_train):
        songs = _user_songs(np.random.default_rng([seed, 1, i]), cdf, perm)
        tr_u.append(np.full(songs.size, i, dtype=np.int64))
        tr_s.append(songs)
    te_u, te_s, lb_u, lb_s = [], [], [], []
    for j in range(test_offset, test_offset + n_test):
        songs = _user_songs(np.random.default_rng([seed, 2, j]), cdf, perm)
        key = n_train + j  # user keys: train 0..n_train-1, then test users
        vis = math.ceil(songs.size / 2)  # NB:571-573
        te_u.append(np.full(vis, key, dtype=np.int64)); te_s.append(songs[:vis])
        lb_u.append(np.full(songs.size - vis, key, dtype=np.int64)); lb_s.append(songs[vis:])
    cat = lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.int64)  # noqa: E731
    return Triplets(cat(tr_u), cat(tr_s), cat(te_u), cat(te_s), cat(lb_u), cat(lb_s), float(alpha))


def calibrate_alpha(n_train: int, n_test: int, seed: int, target_songs: int,
                    n_universe: int = N_SONG_UNIVERSE, tol: float = 0.05) -> float:
    """Bisect alpha (distinct songs decrease with alpha) to within ±tol of target."""
    lo, hi = 0.0, 1.6
    best = None
    for _ in range(30):
        mid = 0.5 * (lo + hi)
        t = generate(n_train, n_test, seed, alpha=mid, n_universe=n_universe)
        ns = t.n_songs()
        err = abs(ns - target_songs) / target_songs
        if best is None or err < best[0]:
            best = (err, mid)
        if err <= tol * 0.2:
            break
        if ns > target_songs:
            lo = mid
        else:
            hi = mid
    return round(best[1], 6)


# Full-scale configs (bulk generator, capped Zipf head; SURVEY.md §8d seeds):
# C4 = the full Taste Profile (1,019,318 users) with the last 10,000 as test
# users; C5 = 2,000 test users against the remaining train set.
BULK_CONFIGS = {
    "c4": (1_009_318, 10_000, 4),
    "c5": (1_017_318, 2_000, 5),
}


def config(name: str, n_test: Optional[int] = None) -> Triplets:
    """Named config; n_test overrides the test-user count (weak-scaling runs
    use n_test = 10 x GPUs with the same train set and the same alpha)."""
    if name in BULK_CONFIGS:
        n_tr, n_te, seed = BULK_CONFIGS[name]
        return generate_bulk(n_tr, n_test if n_test is not None else n_te, seed)
    n_tr, n_te, seed, target = CONFIGS[name]
    alpha = ALPHA.get(name)
    if alpha is None and target is not None:
        alpha = calibrate_alpha(n_tr, n_te, seed, target)
    return generate(n_tr, n_test if n_test is not None else n_te, seed, alpha=alpha)


# ---------------------------------------------------------------------------
# Full-scale generator (C4/C5: ~1M users, ~48M rows). Same distributions as
# ``generate`` but drawn in bulk with numpy (one RNG stream per call, so it is
# NOT prefix-consistent with ``generate``) and with the popularity head capped
# (pure Zipf(0.87) would give the top song more listeners than
# users; the cap keeps every song's expected listener share <= head_cap).
# ---------------------------------------------------------------------------
def capped_popularity(alpha: float, n_universe: int, mean_len: float, head_cap: float) -> np.ndarray:
    """Zipf(alpha) probabilities with water-filling: no song's expected share of
    users (p * mean_len) exceeds head_cap; the excess is spread over the tail."""
    p = np.arange(1, n_universe + 1, dtype=np.float64) ** (-alpha)
    p /= p.sum()
    p_max = head_cap / mean_len
    for _ in range(200):
        over = p > p_max
        if not over.any():
            break
        excess = float((p[over] - p_max).sum())
        p[over] = p_max
        free = ~over & (p < p_max)
        p[free] += excess * p[free] / p[free].sum()
    return p


def generate_bulk(n_train: int, n_test: int, seed: int, alpha: float = 0.87,
                  head_cap: float = 0.10, n_universe: int = N_SONG_UNIVERSE) -> Triplets:
    """Bulk draw of n_train + n_test users (train first, then test), history
    lengths max(10, round(lognormal(3.51, 0.86))), distinct songs by capped
    Zipf popularity in draw order; test users split ceil(n/2) visible / rest
    labels (NB:571-573)."""
    rng = np.random.default_rng([seed, 7])
    n_users = n_train + n_test
    lens = np.maximum(10, np.rint(rng.lognormal(3.51, 0.86, n_users))).astype(np.int64)
    lens = np.minimum(lens, n_universe)
    p = capped_popularity(alpha, n_universe, float(lens.mean()), head_cap)
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    perm = np.random.default_rng([seed, 0]).permutation(n_universe).astype(np.int64)
    # rounds of oversampled draws for the users still short of their length
    got_u = np.zeros(0, np.int64)
    got_s = np.zeros(0, np.int64)
    got_o = np.zeros(0, np.int64)  # global draw order
    have = np.zeros(n_users, np.int64)
    order0 = 0
    for _ in range(64):
        need = lens - have
        short = np.nonzero(need > 0)[0]
        if short.size == 0:
            break
        m = (need[short] * 5) // 4 + 8
        u = np.repeat(short, m)
        r = np.searchsorted(cdf, rng.random(u.size), side="right")
        s = perm[np.minimum(r, n_universe - 1)]
        o = order0 + np.arange(u.size, dtype=np.int64)
        order0 += u.size
        u = np.concatenate([got_u, u]); s = np.concatenate([got_s, s]); o = np.concatenate([got_o, o])
        key = u * n_universe + s
        _, first = np.unique(key, return_index=True)       # first draw of each (user, song)
        u, s, o = u[first], s[first], o[first]
        idx = np.lexsort((o, u))                           # per user, in draw order
        u, s, o = u[idx], s[idx], o[idx]
        start = np.searchsorted(u, np.arange(n_users))
        rank = np.arange(u.size) - start[u]
        keep = rank < lens[u]
        got_u, got_s, got_o = u[keep], s[keep], o[keep]
        have = np.bincount(got_u, minlength=n_users)
    else:
        raise RuntimeError("bulk synthetic draw did not converge")
    start = np.searchsorted(got_u, np.arange(n_users))
    rank = np.arange(got_u.size) - start[got_u]
    is_tr = got_u < n_train
    vis = rank < (lens[got_u] + 1) // 2
    te = ~is_tr & vis
    lb = ~is_tr & ~vis
    return Triplets(got_u[is_tr], got_s[is_tr], got_u[te], got_s[te], got_u[lb], got_s[lb], float(alpha))
