"""oracle/reference_py.py — TEST INFRASTRUCTURE ONLY (never imported by the product).

A pure-Python, line-by-line restatement of the reference Scala class
``MusicRecommender`` (src/main/scala/music_recommandation/MusicRecommender.scala,
"MR") for SMALL inputs: the known-answer test of SURVEY.md §4.2 and the seeded
golden fixtures under tests/golden/. It keeps the reference's data structures
and loop order; only the JVM HashSet iteration order of ``songs`` / ``users``
(MR:28, MR:51) is replaced by first-seen order (summation order: a few ulps).

Parity is NOT pinned by reference outputs (the reference ships no tests or
fixtures and cannot run here: no JVM/scalac/sbt/Spark). It is
pinned by the hand-derived known-answer test of SURVEY.md §4.2, reproduced in
tests/golden/kat.json and checked by tests/test_oracle.py.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

Model = List[Tuple[str, Tuple[str, float]]]


def _split(line: str) -> List[str]:
    """Java ``line split "\\t"``: trailing empty strings are removed."""
    parts = line.split("\t")
    while parts and parts[-1] == "":
        parts.pop()
    return parts


class LiteralRecommender:
    """MR:12-91 — the constructor's ingest, then the models of MR:105-307."""

    def __init__(self, train: Sequence[str], test: Sequence[str], test_labels: Sequence[str]):
        self._mut_songs: Dict[str, None] = {}              # mutSongs (MR:51), insertion order
        self._mut_songs_to_users: Dict[str, List[str]] = {}  # mutSongsToUsersMap (MR:53)
        self.train_users, self.train_map = self._extract(train)   # MR:55
        self.test_users, self.test_map = self._extract(test)      # MR:56
        self.songs: List[str] = list(self._mut_songs)             # MR:58
        self.songs_to_users = dict(self._mut_songs_to_users)      # MR:60-62
        self.test_labels, self.new_songs = self._import_labels(test_labels)  # MR:91

    # MR:26-48
    def _extract(self, lines: Sequence[str]):
        users: Dict[str, None] = {}
        m: Dict[str, List[str]] = {}
        for line in lines:
            f = _split(line.rstrip("\r\n"))
            if len(f) != 3:
                raise ValueError(f"MatchError: {line!r}")  # scala.MatchError (MR:34)
            u, s, _ = f
            users[u] = None
            self._mut_songs[s] = None
            m[u] = [s] + m.get(u, [])                                   # prepend (MR:40)
            self._mut_songs_to_users[s] = [u] + self._mut_songs_to_users.get(s, [])  # MR:41
        return list(users), m

    # MR:70-88
    def _import_labels(self, lines: Sequence[str]):
        labels: Dict[str, List[str]] = {}
        new_songs: Dict[str, None] = {}
        for line in lines:
            f = _split(line.rstrip("\r\n"))
            if len(f) != 3:
                raise ValueError(f"MatchError: {line!r}")
            u, s, _ = f
            new_songs[s] = None
            labels[u] = [s] + labels.get(u, [])
        return labels, list(new_songs)

    # MR:105-111
    def _get_model(self, rank) -> Model:
        out: Model = []
        for s in self.songs:
            for u in self.test_users:
                if s not in self.test_map[u]:
                    out.append((u, (s, rank(u, s))))
        return out

    # MR:132-170
    def get_user_based_model(self) -> Model:
        def cosine(u1: str, u2: str) -> float:
            t, tr = self.test_map[u1], self.train_map[u2]
            num = sum(1 if (song in t and song in tr) else 0 for song in self.songs)
            den = math.sqrt(len(t)) * math.sqrt(len(tr))
            return num / den if den != 0 else 0.0

        def rank(user: str, song: str) -> float:
            acc = 0.0
            for u2 in self.train_users:
                if song in self.train_map[u2]:
                    acc += cosine(user, u2)
            return acc

        return self._get_model(rank)

    # MR:222-261
    def get_item_based_model(self) -> Model:
        def cosine(s1: str, s2: str) -> float:
            l1, l2 = self.songs_to_users[s1], self.songs_to_users[s2]
            num = sum(1 if (v in l1 and v in l2) else 0 for v in self.train_users)
            den = math.sqrt(len(l1)) * math.sqrt(len(l2))
            return num / den if den != 0 else 0.0

        def rank(user: str, song: str) -> float:
            acc = 0.0
            for s2 in self.songs:
                if s2 != song and s2 in self.test_map[user]:
                    acc += cosine(song, s2)
            return acc

        return self._get_model(rank)

    # MR:317-330
    @staticmethod
    def linear_combination(ubm: Model, ibm: Model, alpha: float) -> Model:
        out: Model = []
        for (u1, (s1, r1)), (u2, (s2, r2)) in zip(ubm, ibm):
            if u1 != u2 or s1 != s2:
                raise SystemExit(2)
            out.append((u1, (s1, r1 * alpha + r2 * (1 - alpha))))
        return out

    # MR:361-386
    @staticmethod
    def aggregation(ubm: Model, ibm: Model, item_based_percentage: float = 0.5) -> Model:
        if item_based_percentage < 0 or item_based_percentage > 1:
            raise SystemExit(-1)
        threshold = int(item_based_percentage * len(ubm))
        out: Model = []
        for idx, ((u1, (s1, r1)), (u2, (s2, r2))) in enumerate(zip(ubm, ibm)):
            if u1 != u2 or s1 != s2:
                raise SystemExit(2)
            out.append((u1, (s1, r2)) if idx < threshold else (u1, (s1, r1)))
        return out

    # MR:429-452 with the reference's unseeded java.util.Random replaced by the
    # build's seeded stream (restated here from include/mr_engine.h
    # MR_COMB_STOCHASTIC: 24 bits of splitmix64(seed + (i+1)*golden) / 2^24).
    @staticmethod
    def uniform(seed: int, idx: int) -> float:
        m = (1 << 64) - 1
        z = (seed + (idx + 1) * 0x9E3779B97F4A7C15) & m
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
        z ^= z >> 31
        return (z >> 40) / 16777216.0  # exact in float32 and float64

    @staticmethod
    def stochastic(ubm: Model, ibm: Model, item_based_probability: float = 0.5, seed: int = 0) -> Model:
        if item_based_probability < 0 or item_based_probability > 1:
            raise SystemExit(-1)
        out: Model = []
        for idx, ((u1, (s1, r1)), (u2, (s2, r2))) in enumerate(zip(ubm, ibm)):
            if u1 != u2 or s1 != s2:
                raise SystemExit(2)
            take = LiteralRecommender.uniform(seed, idx) < item_based_probability
            out.append((u1, (s1, r2)) if take else (u1, (s1, r1)))
        return out

    # ---- evaluation, MR:521-639 ----
    @staticmethod
    def prediction_to_class_labels(model: Model, threshold: float) -> Dict[str, List[str]]:
        scores = [el[1][1] for el in model]
        mn, mx = min(scores), max(scores)
        pred: Dict[str, List[str]] = {}
        for u, (s, x) in model:
            den = mx - mn
            v = (x - mn) / den if den != 0 else (math.nan if x - mn == 0 else math.copysign(math.inf, x - mn))
            if v > threshold:  # NaN compares false (MR:529)
                pred[u] = [s] + pred.get(u, [])
        return pred

    def confusion_matrix(self, pred: Dict[str, List[str]], song: str) -> Tuple[int, int, int, int]:
        tp = fp = tn = fn = 0
        for user in self.test_users:
            p = user in pred and song in pred[user]
            lab = song in self.test_labels[user]
            tp += 1 if (p and lab) else 0
            fp += 1 if (p and not lab) else 0
            tn += 1 if ((not p) and not lab) else 0
            fn += 1 if ((not p) and lab) else 0
        return tp, fp, tn, fn

    @staticmethod
    def precision(cm) -> float:
        return cm[0] / (cm[0] + cm[1]) if cm[0] + cm[1] > 0 else 0.0

    @staticmethod
    def recall(cm) -> float:
        return cm[0] / (cm[0] + cm[3]) if cm[0] + cm[3] > 0 else 0.0

    THRESHOLDS = [0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9]  # MR:590
    THRESHOLDS_DISTRIBUTED = [0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9, 1.0]  # distributed.scala:395

    def average_precision(self, model: Model, thresholds=None) -> List[Tuple[str, float]]:
        """MR:588-618 (thresholds=None); with THRESHOLDS_DISTRIBUTED the same
        recurrence over 11 thresholds, distributed.scala:394-416."""
        ths = self.THRESHOLDS if thresholds is None else thresholds
        preds = [self.prediction_to_class_labels(model, t) for t in ths]
        out = []
        for song in self.new_songs:
            terms = []
            for i, _t in enumerate(ths):
                if i == len(ths) - 1:
                    terms.append(0.0)
                elif i == len(ths) - 2:
                    cm = self.confusion_matrix(preds[i], song)
                    terms.append((self.recall(cm) - 0.0) * self.precision(cm))
                else:
                    cm = self.confusion_matrix(preds[i], song)
                    cm1 = self.confusion_matrix(preds[i + 1], song)
                    terms.append((self.recall(cm) - self.recall(cm1)) * self.precision(cm))
            acc = 0.0
            for x in terms:  # List.sum = left fold
                acc += x
            out.append((song, acc))
        return out

    def evaluate_model(self, model: Model, thresholds=None) -> float:
        """MR:625-639 (foldLeft over newSongs); distributed.scala:424-442 sums
        with RDD.sum (partition order) over the same values."""
        acc = 0.0
        for _s, ap in self.average_precision(model, thresholds):
            acc += ap
        return acc / len(self.new_songs)


def map_at_k(model: Model, test_labels: Dict[str, List[str]], test_users: Sequence[str], k: int = 10) -> float:
    """Build-defined mAP@k (the reference has none): per test
    user, rank its unheard songs by (score desc, song id asc), then
    AP@k = Σ_{i<=k} P@i·rel(i) / min(k, |labels(u)|), mean over test users."""
    per: Dict[str, List[Tuple[float, str]]] = {}
    for u, (s, x) in model:
        per.setdefault(u, []).append((x, s))
    total = 0.0
    for u in test_users:
        labels = set(test_labels.get(u, []))
        cands = sorted(per.get(u, []), key=lambda t: (-t[0], t[1]))[:k]
        hits = 0
        ap = 0.0
        for i, (_x, s) in enumerate(cands, start=1):
            if s in labels:
                hits += 1
                ap += hits / i
        denom = min(k, len(labels))
        total += ap / denom if denom > 0 else 0.0
    return total / len(test_users) if test_users else 0.0
