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


def label_matrix(ds: Dataset) -> np.ndarray:
    m = np.zeros((ds.n_test, ds.n_songs), dtype=bool)
    rows = np.repeat(np.arange(ds.n_test), np.diff(ds.lab_off))
    keep = ds.lab_songs < ds.n_songs          # label-only songs are never predicted
    m[rows[keep], ds.lab_songs[keep]] = True
    return m


def threshold_map(scores: np.ndarray, ds: Dataset, thresholds=THRESHOLDS) -> float:
    """Reference threshold mAP of a dense model (MR:636)."""
    x = np.asarray(scores, dtype=np.float64)
    valid = ~np.isnan(x)
    if ds.n_label_songs == 0:
        return float("nan")
    mn = x[valid].min()
    mx = x[valid].max()
    with np.errstate(invalid="ignore", divide="ignore"):
        norm = (x - mn) / (mx - mn)
    lab = label_matrix(ds)
    pos = lab.sum(axis=0)                      # TP + FN per song
    P, R = [], []
    for t in thresholds:
        with np.errstate(invalid="ignore"):
            pred = valid & (norm > t)          # NaN > t is False (MR:529)
        tp = (pred & lab).sum(axis=0)
        pp = pred.sum(axis=0)                  # TP + FP
        P.append(np.where(pp > 0, tp / np.maximum(pp, 1), 0.0))
        R.append(np.where(pos > 0, tp / np.maximum(pos, 1), 0.0))
    n = len(thresholds)
    ap = np.zeros(ds.n_songs)
    for i in range(n):                         # List.sum: left fold in threshold order
        if i == n - 1:
            term = 0.0
        elif i == n - 2:
            term = (R[i] - 0.0) * P[i]
        else:
            term = (R[i] - R[i + 1]) * P[i]
        ap = ap + term
    cls = pos > 0                              # other newSongs have AP = 0
    total = 0.0
    for v in ap[cls]:
        total += float(v)
    return total / ds.n_label_songs


def map_at_k(top_songs: np.ndarray, ds: Dataset, k: int = 10) -> float:
    """Build-defined mAP@k of per-user top-k lists (song -1 = empty slot)."""
    total = 0.0
    for u in range(ds.n_test):
        labels = set(ds.lab_songs[ds.lab_off[u]:ds.lab_off[u + 1]].tolist())
        hits = 0
        ap = 0.0
        for i, s in enumerate(top_songs[u, :k].tolist(), start=1):
            if s >= 0 and s in labels:
                hits += 1
                ap += hits / i
        denom = min(k, len(labels))
        total += ap / denom if denom else 0.0
    return total / ds.n_test if ds.n_test else 0.0
