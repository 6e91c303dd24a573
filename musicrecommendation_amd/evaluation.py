"""Model quality over engine outputs (host side; the scores come from the GPU).

* ``threshold_map`` — the reference's evaluateModel (MusicRecommender.scala
  MR:521-639): global min/max normalisation (MR:524-525), prediction if the
  normalised score is > t for t in 0.0..0.9 (MR:529, MR:590), per new-song
  confusion over the test users (MR:541-553), AP(g) = Σ_{i<8} (R_i−R_{i+1})·P_i
  + R_8·P_8 + 0 (MR:601-609), mAP = Σ AP / |newSongs| (MR:626).
* ``map_at_k`` — the build-defined mAP@k over the engine's top-k lists
  (SURVEY.md §8d): AP@k(u) = Σ_{i<=k} P@i·rel(i) / min(k, |labels(u)|).
Vectorised over the dense n_test x n_songs score matrix (NaN = no pair).
"""
from __future__ import annotations

import numpy as np

from .dataset import Dataset

THRESHOLDS = (0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9)  # MR:590
# the distributed evaluation's 11 thresholds (distributed.scala:395)
THRESHOLDS_DISTRIBUTED = THRESHOLDS + (1.0,)


def label_matrix(ds: Dataset) -> np.ndarray:
    m = np.zeros((ds.n_test, ds.n_songs), dtype=bool)
    rows = np.repeat(np.arange(ds.n_test), np.diff(ds.lab_off))
    keep = ds.lab_songs < ds.n_songs          # label-only songs are never predicted
    m[rows[keep], ds.lab_songs[keep]] = True
    return m


def label_pos(ds: Dataset) -> np.ndarray:
    """pos[s] = #test users whose labels hold song s (TP + FN of class s), s < n_songs."""
    keep = ds.lab_songs < ds.n_songs
    return np.bincount(ds.lab_songs[keep], minlength=ds.n_songs).astype(np.int32)


def threshold_counts(scores: np.ndarray, ds: Dataset, mn: float, mx: float, thresholds=THRESHOLDS):
    """(pred, tp), each n_songs x len(thresholds): per song and threshold, the test users
    predicted ((x - mn)/(mx - mn) > t, MR:529) and those of them whose labels
    hold the song (MR:541-553). The numpy twin of mr_eval_counts_device."""
    x = np.asarray(scores, dtype=np.float64)
    valid = ~np.isnan(x)
    with np.errstate(invalid="ignore", divide="ignore"):
        norm = (x - mn) / (mx - mn)
    lab = label_matrix(ds)
    pred = np.zeros((x.shape[1], len(thresholds)), dtype=np.int64)
    tp = np.zeros_like(pred)
    for i, t in enumerate(thresholds):
        with np.errstate(invalid="ignore"):
            p = valid & (norm > t)             # NaN > t is False (MR:529)
        pred[:, i] = p.sum(axis=0)
        tp[:, i] = (p & lab).sum(axis=0)
    return pred, tp


def map_from_counts(pred: np.ndarray, tp: np.ndarray, pos: np.ndarray, n_label_songs: int) -> float:
    """AP per class (MR:588-618) and the mean (MR:625-627) from the counts:
    P_i = TP/(TP+FP), R_i = TP/(TP+FN) (MR:563-581), with n = pred.shape[1]
    thresholds AP = Σ_{i<n-2} (R_i−R_{i+1})·P_i + R_{n-2}·P_{n-2} + 0 (left
    fold; n = 10 MR:601-609, n = 11 distributed.scala:405-413), classes summed
    in song-id order."""
    if n_label_songs == 0:
        return float("nan")
    pred = np.asarray(pred, dtype=np.float64)
    tp = np.asarray(tp, dtype=np.float64)
    pos = np.asarray(pos)
    n = pred.shape[1]
    P = [np.where(pred[:, i] > 0, tp[:, i] / np.maximum(pred[:, i], 1), 0.0) for i in range(n)]
    R = [np.where(pos > 0, tp[:, i] / np.maximum(pos, 1), 0.0) for i in range(n)]
    ap = np.zeros(pred.shape[0])
    for i in range(n):                         # List.sum: left fold in threshold order
        if i == n - 1:
            term = 0.0
        elif i == n - 2:
            term = (R[i] - 0.0) * P[i]
        else:
            term = (R[i] - R[i + 1]) * P[i]
        ap = ap + term
    total = 0.0
    for v in ap[pos > 0]:                      # other newSongs have AP = 0
        total += float(v)
    return total / n_label_songs


def threshold_map(scores: np.ndarray, ds: Dataset, thresholds=THRESHOLDS) -> float:
    """Reference threshold mAP of a dense model (MR:636), on the host."""
    x = np.asarray(scores, dtype=np.float64)
    valid = ~np.isnan(x)
    if ds.n_label_songs == 0:
        return float("nan")
    mn = x[valid].min()
    mx = x[valid].max()
    pred, tp = threshold_counts(x, ds, mn, mx, thresholds)
    return map_from_counts(pred, tp, label_pos(ds), ds.n_label_songs)


def map_at_k(top_songs: np.ndarray, ds: Dataset, k: int = 10) -> float:
    """Build-defined mAP@k of per-user top-k lists (song -1 = empty slot):
    per test user, Σ_i hit_i · (hits up to i) / i over the first k slots,
    divided by min(k, |distinct labels|); users without labels count 0.
    Vectorised: membership of every (user, song) slot in the user's label set
    by one binary search over the sorted (user, song) label keys."""
    n_te = ds.n_test
    if n_te == 0:
        return 0.0
    top = np.asarray(top_songs)[:, :k].astype(np.int64)
    lab_off = np.asarray(ds.lab_off, dtype=np.int64)
    lab = np.asarray(ds.lab_songs, dtype=np.int64)
    m = int(max(int(lab.max()) if lab.size else 0, int(top.max()) if top.size else 0)) + 1
    lab_user = np.repeat(np.arange(n_te, dtype=np.int64), np.diff(lab_off))
    keys = np.unique(lab_user * m + lab)  # distinct labels per user (set semantics)
    n_lab = np.bincount(keys // m, minlength=n_te)
    q = np.arange(n_te, dtype=np.int64)[:, None] * m + np.maximum(top, 0)
    pos = np.minimum(np.searchsorted(keys, q), max(keys.size - 1, 0))
    hit = (top >= 0) & (keys.size > 0) & (keys[pos] == q) if keys.size else np.zeros_like(top, dtype=bool)
    ranks = np.arange(1, top.shape[1] + 1, dtype=np.float64)
    ap = (hit * (np.cumsum(hit, axis=1) / ranks)).sum(axis=1)
    denom = np.minimum(k, n_lab)
    return float(np.where(denom > 0, ap / np.maximum(denom, 1), 0.0).sum() / n_te)
