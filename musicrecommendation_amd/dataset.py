"""Interned dataset: the engine's input (mr_dataset of include/mr_engine.h).

Two constructors, with identical semantics (checked by tests/test_ingest.py):
  * ``Dataset.from_tsv``      — the native C++ ingest (mr_corpus_from_tsv), the
                                replacement of extractData/importTestLabels
                                (MusicRecommender.scala MR:26-91);
  * ``Dataset.from_triplets`` — numpy build from integer-keyed triplets (the
                                synthetic generator's output) whose names sort
                                like their integer keys.

Semantics kept from the reference:
  songs        = distinct songs of train ∪ test (labels add none, MR:58/79)
  song_count   = songsToUsersMap(s).length: train + test lines, duplicates counted
  tr_len/te_len = per-user `.length` with duplicates (MR:147)
  CSR rows     = sorted, duplicate-free song ids (`contains` is a set test)
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence

import numpy as np

from . import _lib


def song_name(key: int) -> str:
    """Synthetic song id: 18 chars like the Taste Profile's (e.g. SOAKIMP12A8C130995).
    Fixed-width upper-case hex keeps lexicographic order == numeric order."""
    return "SO%016X" % key


def user_name(key: int) -> str:
    """Synthetic user id: 40 lower-case hex chars (the Taste Profile's SHA-1 width)."""
    return "%040x" % key


class _Corpus:
    """Owner of a native mr_corpus: freed when the last array viewing it dies."""

    def __init__(self, L, h):
        self._L, self._h = L, h

    def __del__(self):  # pragma: no cover - interpreter-driven
        try:
            if self._h:
                self._L.mr_corpus_free(self._h)
        except Exception:
            pass

    def view(self, addr, n: int, dt) -> np.ndarray:
        if n == 0 or not addr:
            return np.zeros(0, dtype=dt)
        return np.asarray(_Buffer(self, addr, n, np.dtype(dt)))

    def names(self, kind: int, n: int) -> "_Names":
        need = ctypes.c_int64()
        _lib.check(self._L.mr_corpus_names(self._h, kind, None, 0, ctypes.byref(need)), "mr_corpus_names")
        buf = np.empty(max(1, need.value), dtype=np.uint8)
        _lib.check(self._L.mr_corpus_names(self._h, kind, buf.ctypes.data_as(ctypes.c_char_p), need.value,
                                           ctypes.byref(need)), "mr_corpus_names")
        ends = np.flatnonzero(buf[:need.value] == 10)
        if ends.size != n:
            raise RuntimeError(f"mr_corpus_names: {ends.size} names of kind {kind}, expected {n}")
        return _Names(buf, ends)


class _Buffer:
    """Read-only numpy view of native memory that keeps its owner alive (the
    array's base). Read-only: the corpus is shared by every view, so an
    in-place edit would silently change them all — copy first to modify."""

    def __init__(self, owner, addr: int, n: int, dt: np.dtype):
        self._owner = owner
        self.__array_interface__ = {"shape": (n,), "typestr": dt.str, "data": (addr, True), "version": 3}


class _Names:
    """Names of one kind, newline-separated in one buffer; decoded on access."""

    def __init__(self, buf: np.ndarray, ends: np.ndarray):
        self._buf, self._ends = buf, ends

    def __len__(self) -> int:
        return int(self._ends.size)

    def __getitem__(self, i: int) -> str:
        i = int(i)
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        a = int(self._ends[i - 1]) + 1 if i else 0
        return self._buf[a:int(self._ends[i])].tobytes().decode()


@dataclass
class Dataset:
    n_train: int
    n_test: int
    n_songs: int
    tr_off: np.ndarray      # int64 [n_train+1]
    tr_songs: np.ndarray    # int32
    te_off: np.ndarray      # int64 [n_test+1]
    te_songs: np.ndarray    # int32
    song_count: np.ndarray  # int32 [n_songs]
    tr_len: np.ndarray      # int32 [n_train]
    te_len: np.ndarray      # int32 [n_test]
    lab_off: np.ndarray     # int64 [n_test+1] labels over test users
    lab_songs: np.ndarray   # int32; ids >= n_songs are label-only songs
    n_label_songs: int      # distinct songs of the labels file (newSongs, MR:79)
    n_extra_songs: int = 0  # label-only songs (ids n_songs .. n_songs+n_extra-1)
    song_names: Optional[Callable[[int], str]] = None
    train_names: Optional[Callable[[int], str]] = None
    test_names: Optional[Callable[[int], str]] = None
    _keep: list = field(default_factory=list, repr=False)

    # ---- views -------------------------------------------------------------
    def c_struct(self) -> _lib.MrDataset:
        arrs = [
            np.ascontiguousarray(self.tr_off, dtype=np.int64),
            np.ascontiguousarray(self.tr_songs, dtype=np.int32),
            np.ascontiguousarray(self.te_off, dtype=np.int64),
            np.ascontiguousarray(self.te_songs, dtype=np.int32),
            np.ascontiguousarray(self.song_count, dtype=np.int32),
            np.ascontiguousarray(self.tr_len, dtype=np.int32),
            np.ascontiguousarray(self.te_len, dtype=np.int32),
        ]
        self._keep = arrs
        P64 = ctypes.POINTER(ctypes.c_int64)
        P32 = ctypes.POINTER(ctypes.c_int32)
        d = _lib.MrDataset()
        d.n_train_users, d.n_test_users, d.n_songs = self.n_train, self.n_test, self.n_songs
        d.tr_off = arrs[0].ctypes.data_as(P64)
        d.tr_songs = arrs[1].ctypes.data_as(P32)
        d.te_off = arrs[2].ctypes.data_as(P64)
        d.te_songs = arrs[3].ctypes.data_as(P32)
        d.song_count = arrs[4].ctypes.data_as(P32)
        d.tr_len = arrs[5].ctypes.data_as(P32)
        d.te_len = arrs[6].ctypes.data_as(P32)
        return d

    def heard_mask(self) -> np.ndarray:
        """Boolean n_test x n_songs: song in T(u) (no pair emitted, MR:109)."""
        m = np.zeros((self.n_test, self.n_songs), dtype=bool)
        rows = np.repeat(np.arange(self.n_test), np.diff(self.te_off))
        m[rows, self.te_songs] = True
        return m

    def n_pairs(self) -> int:
        """P = Σ_u (n_s − |T(u) ∩ songs|): the number of scored pairs (MR:105-111)."""
        return int(self.n_test) * int(self.n_songs) - int(self.te_off[-1])

    def subset_test_users(self, lo: int, hi: int) -> "Dataset":
        """Test users [lo, hi) against the same train data, songs and counts.
        c(s) keeps every test user's listens (MR:60-62), so each user's
        scores are exactly those of the full dataset: a partition of the
        model's pairs by test user."""
        a, b = int(self.te_off[lo]), int(self.te_off[hi])
        la, lb = int(self.lab_off[lo]), int(self.lab_off[hi])
        base_names = self.test_names
        return Dataset(
            n_train=self.n_train, n_test=hi - lo, n_songs=self.n_songs,
            tr_off=self.tr_off, tr_songs=self.tr_songs,
            te_off=self.te_off[lo:hi + 1] - a, te_songs=self.te_songs[a:b],
            song_count=self.song_count, tr_len=self.tr_len, te_len=self.te_len[lo:hi],
            lab_off=self.lab_off[lo:hi + 1] - la, lab_songs=self.lab_songs[la:lb],
            n_label_songs=self.n_label_songs, n_extra_songs=self.n_extra_songs,
            song_names=self.song_names, train_names=self.train_names,
            test_names=(lambda i: base_names(lo + i)) if base_names else None,
        )

    def label_sets(self) -> List[np.ndarray]:
        return [self.lab_songs[self.lab_off[u]:self.lab_off[u + 1]] for u in range(self.n_test)]

    # ---- constructors --------------------------------------------------------
    @staticmethod
    def from_tsv(train_path: str, test_path: str, labels_path: Optional[str] = None) -> "Dataset":
        """Native ingest (mr_corpus_from_tsv). The arrays are views of the
        native corpus (no copy), which lives as long as any of them."""
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(
            L.mr_corpus_from_tsv(
                os.fsencode(train_path), os.fsencode(test_path),
                os.fsencode(labels_path) if labels_path else None, ctypes.byref(h)),
            "mr_corpus_from_tsv")
        owner = _Corpus(L, h)
        d = _lib.MrDataset()
        _lib.check(L.mr_corpus_dataset(h, ctypes.byref(d)), "mr_corpus_dataset")
        n_tr, n_te, n_s = d.n_train_users, d.n_test_users, d.n_songs

        def arr(ptr, n, dt):
            return owner.view(ctypes.cast(ptr, ctypes.c_void_p).value, n, dt)

        tr_off = arr(d.tr_off, n_tr + 1, np.int64)
        te_off = arr(d.te_off, n_te + 1, np.int64)
        lo = ctypes.POINTER(ctypes.c_int64)()
        ls = ctypes.POINTER(ctypes.c_int32)()
        nl = ctypes.c_int32()
        ne = ctypes.c_int32()
        _lib.check(L.mr_corpus_labels(h, ctypes.byref(lo), ctypes.byref(ls), ctypes.byref(nl), ctypes.byref(ne)),
                   "mr_corpus_labels")
        lab_off = arr(lo, n_te + 1, np.int64)
        names_s = owner.names(0, n_s + ne.value)
        names_tr = owner.names(1, n_tr)
        names_te = owner.names(2, n_te)
        return Dataset(
            n_train=n_tr, n_test=n_te, n_songs=n_s,
            tr_off=tr_off, tr_songs=arr(d.tr_songs, int(tr_off[-1]), np.int32),
            te_off=te_off, te_songs=arr(d.te_songs, int(te_off[-1]), np.int32),
            song_count=arr(d.song_count, n_s, np.int32),
            tr_len=arr(d.tr_len, n_tr, np.int32), te_len=arr(d.te_len, n_te, np.int32),
            lab_off=lab_off, lab_songs=arr(ls, int(lab_off[-1]), np.int32),
            n_label_songs=nl.value, n_extra_songs=ne.value,
            song_names=names_s.__getitem__, train_names=names_tr.__getitem__,
            test_names=names_te.__getitem__,
        )

    @staticmethod
    def from_triplets(train_u: np.ndarray, train_s: np.ndarray, test_u: np.ndarray, test_s: np.ndarray,
                      label_u: Optional[np.ndarray] = None, label_s: Optional[np.ndarray] = None,
                      song_name_fn: Callable[[int], str] = song_name,
                      user_name_fn: Callable[[int], str] = user_name) -> "Dataset":
        """Integer-keyed triplets -> dataset. Keys are interned in ascending
        order, which must equal the lexicographic order of their names (true
        for song_name/user_name above)."""
        train_u = np.asarray(train_u, dtype=np.int64)
        train_s = np.asarray(train_s, dtype=np.int64)
        test_u = np.asarray(test_u, dtype=np.int64)
        test_s = np.asarray(test_s, dtype=np.int64)
        tr_keys = np.unique(train_u)
        te_keys = np.unique(test_u)
        if np.intersect1d(tr_keys, te_keys).size:
            raise ValueError("train and test users overlap")
        song_keys = np.unique(np.concatenate([train_s, test_s]))
        n_s = song_keys.size
        tu = np.searchsorted(tr_keys, train_u)
        ts = np.searchsorted(song_keys, train_s)
        eu = np.searchsorted(te_keys, test_u)
        es = np.searchsorted(song_keys, test_s)
        song_count = (np.bincount(ts, minlength=n_s) + np.bincount(es, minlength=n_s)).astype(np.int32)

        def csr(rows, cols, n_rows):
            ln = np.bincount(rows, minlength=n_rows).astype(np.int32)
            key = np.unique(rows.astype(np.int64) * (1 << 32) + cols)
            r = (key >> 32).astype(np.int64)
            c = (key & 0xFFFFFFFF).astype(np.int32)
            off = np.zeros(n_rows + 1, dtype=np.int64)
            np.cumsum(np.bincount(r, minlength=n_rows), out=off[1:])
            return off, c, ln

        tr_off, tr_songs, tr_len = csr(tu, ts, tr_keys.size)
        te_off, te_songs, te_len = csr(eu, es, te_keys.size)
        # labels
        n_extra = 0
        if label_u is not None and len(label_u):
            label_u = np.asarray(label_u, dtype=np.int64)
            label_s = np.asarray(label_s, dtype=np.int64)
            all_label_songs = np.unique(label_s)
            n_label = all_label_songs.size
            keep = np.isin(label_u, te_keys)
            lu = np.searchsorted(te_keys, label_u[keep])
            ls_keys = label_s[keep]
            in_songs = np.isin(ls_keys, song_keys)
            extra_keys = np.setdiff1d(all_label_songs, song_keys)
            n_extra = extra_keys.size
            lid = np.where(in_songs, np.searchsorted(song_keys, ls_keys),
                           n_s + np.searchsorted(extra_keys, ls_keys))
            key = np.unique(lu.astype(np.int64) * (1 << 32) + lid)
            r = key >> 32
            lab_songs = (key & 0xFFFFFFFF).astype(np.int32)
            lab_off = np.zeros(te_keys.size + 1, dtype=np.int64)
            np.cumsum(np.bincount(r, minlength=te_keys.size), out=lab_off[1:])
            all_song_keys = np.concatenate([song_keys, extra_keys])
        else:
            n_label = 0
            lab_off = np.zeros(te_keys.size + 1, dtype=np.int64)
            lab_songs = np.zeros(0, dtype=np.int32)
            all_song_keys = song_keys
        return Dataset(
            n_train=int(tr_keys.size), n_test=int(te_keys.size), n_songs=int(n_s),
            tr_off=tr_off, tr_songs=tr_songs, te_off=te_off, te_songs=te_songs,
            song_count=song_count, tr_len=tr_len, te_len=te_len,
            lab_off=lab_off, lab_songs=lab_songs, n_label_songs=int(n_label), n_extra_songs=int(n_extra),
            song_names=lambda i: song_name_fn(int(all_song_keys[i])),
            train_names=lambda i: user_name_fn(int(tr_keys[i])),
            test_names=lambda i: user_name_fn(int(te_keys[i])),
        )

    # ---- arrays on disk (one build shared by the ranks of a node) --------------
    _ARRAYS = ("tr_off", "tr_songs", "te_off", "te_songs", "song_count", "tr_len", "te_len", "lab_off", "lab_songs")

    def save_arrays(self, path: str) -> None:
        """The interned arrays as one uncompressed .npz (names are not kept):
        bench.py's multi-rank runs build the full-scale dataset once and the
        other ranks of the node load it (Dataset.load_arrays)."""
        sizes = np.array([self.n_train, self.n_test, self.n_songs, self.n_label_songs, self.n_extra_songs],
                         dtype=np.int64)
        np.savez(path, sizes=sizes, **{k: np.asarray(getattr(self, k)) for k in self._ARRAYS})

    @staticmethod
    def load_arrays(path: str) -> "Dataset":
        """Dataset.save_arrays' file -> Dataset without names (no pickles:
        allow_pickle=False)."""
        with np.load(path, allow_pickle=False) as z:
            n_tr, n_te, n_s, n_lab, n_extra = (int(x) for x in z["sizes"])
            arrs = {k: z[k] for k in Dataset._ARRAYS}
        return Dataset(n_train=n_tr, n_test=n_te, n_songs=n_s, n_label_songs=n_lab, n_extra_songs=n_extra, **arrs)

    # ---- export ---------------------------------------------------------------
    def write_tsv(self, train_path: str, test_path: str, labels_path: str) -> None:
        """Write the dataset as reference-format triplet files (playcount 1).
        Duplicate lines are not reproduced (the CSR keeps sets); use this for
        duplicate-free datasets only."""
        for path, off, col, names in ((train_path, self.tr_off, self.tr_songs, self.train_names),
                                      (test_path, self.te_off, self.te_songs, self.test_names),
                                      (labels_path, self.lab_off, self.lab_songs, self.test_names)):
            with open(path, "w") as f:
                for u in range(len(off) - 1):
                    un = names(u)
                    for s in col[off[u]:off[u + 1]]:
                        f.write(f"{un}\t{self.song_names(int(s))}\t1\n")
