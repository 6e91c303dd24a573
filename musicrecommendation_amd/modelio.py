"""Model files of the reference (MusicRecommender.scala MR:489-512), through the
engine library's host code (csrc/mr_modelio.cpp):

* ``write_dense`` — writeModelOnFile (MR:489-497) of a dense model: one
  ``user\\tsong\\tscore`` line per pair, scores as java.lang.Double.toString;
* ``read_dense``  — importModelFromFile (MR:505-512) into a dense model over a
  dataset's interned names (NaN where the file has no pair);
* ``java_double_string`` — Scala's ``s"${x}"`` of a Double.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Tuple

import numpy as np

from . import _lib
from .dataset import Dataset


def java_double_string(x: float) -> str:
    buf = ctypes.create_string_buffer(40)
    n = _lib.lib().mr_java_double_string(float(x), buf, 40)
    if n < 0:
        _lib.check(n, "mr_java_double_string")
    return buf.value.decode()


def _names(fn, n: int):
    arr = (ctypes.c_char_p * max(1, n))()
    keep = [fn(i).encode() for i in range(n)]
    for i, b in enumerate(keep):
        arr[i] = b
    return arr, keep


def write_dense(path: str, ds: Dataset, dense: np.ndarray, order: str = "sorted") -> None:
    """order 'emission' = getModel's song-major enumeration (MR:106-108);
    'sorted' = the driver's (user, song) order (main.scala:57-59)."""
    d = np.ascontiguousarray(dense, dtype=np.float64)
    if d.shape != (ds.n_test, ds.n_songs):
        raise ValueError(f"dense model shape {d.shape} != ({ds.n_test}, {ds.n_songs})")
    users, ku = _names(ds.test_names, ds.n_test)
    songs, ks = _names(ds.song_names, ds.n_songs)
    _lib.check(_lib.lib().mr_model_write_tsv(os.fsencode(path), ds.n_test, ds.n_songs, users, songs,
                                             d.ctypes.data_as(ctypes.c_void_p), {"emission": 0, "sorted": 1}[order]),
               "mr_model_write_tsv")


def read_dense(path: str, ds: Dataset) -> np.ndarray:
    out = np.empty((ds.n_test, ds.n_songs), dtype=np.float64)
    users, ku = _names(ds.test_names, ds.n_test)
    songs, ks = _names(ds.song_names, ds.n_songs)
    _lib.check(_lib.lib().mr_model_read_tsv(os.fsencode(path), ds.n_test, ds.n_songs, users, songs,
                                            out.ctypes.data_as(ctypes.c_void_p)), "mr_model_read_tsv")
    return out


def import_model(path: str) -> List[Tuple[str, str, float]]:
    """importModelFromFile (MR:505-512) as the reference returns it: triplets
    sorted by (user, song, -score). Malformed lines raise ValueError (the
    reference: scala.MatchError / NumberFormatException)."""
    rows = []
    with open(path) as f:
        for n, line in enumerate(f, start=1):
            parts = line.rstrip("\r\n").split("\t")
            while parts and parts[-1] == "":
                parts.pop()
            if len(parts) != 3:
                raise ValueError(f"{path}:{n}: MatchError: expected 3 tab-separated fields")
            rows.append((parts[0], parts[1], float(parts[2])))
    rows.sort(key=lambda t: (t[0], t[1], -t[2]))
    return rows
