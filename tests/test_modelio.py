"""Model files (MR:489-512) on the host: java.lang.Double.toString formatting,
dense write -> read round trips in both line orders, the reference's
importModelFromFile ordering, and the error codes for malformed files."""
import math
import os
import random
import struct

import numpy as np
import pytest

from musicrecommendation_amd import _lib
from musicrecommendation_amd.modelio import import_model, java_double_string, read_dense, write_dense
from musicrecommendation_amd.recommender import MusicRecommender

from helpers import synth_fixture

# Outputs of java.lang.Double.toString (JDK 19+ javadoc examples and classic cases)
KNOWN = [
    (1.0, "1.0"), (0.001, "0.001"), (1e-4, "1.0E-4"), (1e7, "1.0E7"), (1234567.0, "1234567.0"),
    (12345678.0, "1.2345678E7"), (0.1 + 0.2, "0.30000000000000004"), (100.0, "100.0"), (2 / 3, "0.6666666666666666"),
    (-3.5, "-3.5"), (0.0, "0.0"), (-0.0, "-0.0"), (2e23, "2.0E23"), (5e-324, "4.9E-324"),
    (1.7976931348623157e308, "1.7976931348623157E308"), (float("nan"), "NaN"), (float("inf"), "Infinity"),
    (float("-inf"), "-Infinity"), (0.40824829046386296, "0.40824829046386296"), (1e21, "1.0E21"),
    (9.999999999999999e-4, "9.999999999999998E-4"),
    (2.0 ** -24, "5.960464477539063E-8"),  # asymmetric rounding interval
]


def test_java_double_known_values():
    for x, s in KNOWN:
        if x != x:
            assert java_double_string(x) == "NaN"
            continue
        assert java_double_string(x) == s, (x, java_double_string(x), s)


def _digits(s):
    m = s.lstrip("-").split("E")[0].replace(".", "").lstrip("0").rstrip("0")
    return m or "0"


def test_java_double_random_round_trip_and_shortest():
    rng = random.Random(1)
    for _ in range(20000):
        x = struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0]
        if not math.isfinite(x) or x == 0:
            continue
        s = java_double_string(x)
        assert float(s) == x
        a = abs(x)
        assert ("E" in s) == (not (1e-3 <= a < 1e7))
        if "E" not in s:
            assert "." in s and not s.endswith(".")
        shortest = len(_digits(repr(x).replace("e", "E")))  # Python repr = shortest round trip
        assert len(_digits(s)) <= max(shortest, 2)
        assert len(_digits(s)) >= shortest or shortest == 1


def test_java_double_powers_of_two_shortest_closest():
    """At powers of two the rounding interval is asymmetric: the correctly
    rounded p-digit decimal can miss while its neighbour reads back. Digits
    must equal Python's repr (shortest, then closest: the JDK 19+ rule) for
    every binade, apart from the 1-digit special case."""
    for k in range(-1074, 1024):
        x = math.ldexp(1.0, k)
        s = java_double_string(x)
        assert float(s) == x, (k, s)
        ref = _digits(repr(x).replace("e", "E"))
        if len(ref) >= 2:
            assert _digits(s) == ref, (k, s, repr(x))


@pytest.mark.parametrize("order", ["sorted", "emission"])
def test_dense_round_trip(tmp_path, order):
    ds, z = synth_fixture("small")
    dense = z["ibm"]
    p = str(tmp_path / "m.txt")
    write_dense(p, ds, dense, order)
    lines = open(p).read().splitlines()
    assert len(lines) == int((~np.isnan(dense)).sum())
    got = read_dense(p, ds)
    assert np.array_equal(got.view(np.int64)[~np.isnan(dense)], dense.view(np.int64)[~np.isnan(dense)])
    assert np.isnan(got[np.isnan(dense)]).all()
    first = lines[0].split("\t")
    if order == "sorted":
        assert (first[0], first[1]) == (ds.test_names(0), ds.song_names(int(np.flatnonzero(~np.isnan(dense[0]))[0])))
    else:
        s0 = int(np.flatnonzero((~np.isnan(dense)).any(axis=0))[0])
        assert first[1] == ds.song_names(s0)
    tri = import_model(p)
    assert tri == sorted(tri, key=lambda t: (t[0], t[1], -t[2]))
    assert len(tri) == len(lines)


def test_list_api_matches_dense_writer(tmp_path):
    ds, z = synth_fixture("tiny")
    dense = z["ubm"]
    model = [(ds.test_names(u), (ds.song_names(s), float(dense[u, s])))
             for u in range(ds.n_test) for s in range(ds.n_songs) if not np.isnan(dense[u, s])]
    a, b = str(tmp_path / "a.txt"), str(tmp_path / "b.txt")
    MusicRecommender.writeModelOnFile(model, a)
    write_dense(b, ds, dense, "sorted")
    assert open(a).read() == open(b).read()
    assert MusicRecommender.importModelFromFile(a) == import_model(b)


def test_malformed_files(tmp_path):
    ds, z = synth_fixture("tiny")
    p = str(tmp_path / "bad.txt")
    u, s = ds.test_names(0), ds.song_names(0)
    for text, code in ((f"{u}\t{s}\n", _lib.MR_E_PARSE), (f"{u}\t{s}\tabc\n", _lib.MR_E_PARSE),
                       (f"nobody\t{s}\t1.0\n", _lib.MR_E_INVALID),
                       (f"{u}\t{s}\t1.0\n{u}\t{s}\t2.0\n", _lib.MR_E_INVALID)):
        with open(p, "w") as f:
            f.write(text)
        with pytest.raises(_lib.EngineError) as ei:
            read_dense(p, ds)
        assert ei.value.code == code
    with pytest.raises(_lib.EngineError) as ei:
        read_dense(str(tmp_path / "missing.txt"), ds)
    assert ei.value.code == _lib.MR_E_IO
