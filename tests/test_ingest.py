"""Native TSV ingest (mr_corpus_from_tsv) vs the reference's extractData /
importTestLabels semantics (MusicRecommender.scala MR:26-91). CPU only."""
import os

import numpy as np
import pytest

from musicrecommendation_amd import _lib, synth
from musicrecommendation_amd.dataset import Dataset
from oracle import native

from helpers import dataset_from_lines, kat


def test_kat_corpus_semantics():
    K = kat()
    ds = dataset_from_lines(K["train"], K["test"], K["labels"])
    names = [ds.song_names(i) for i in range(ds.n_songs + ds.n_extra_songs)]
    assert names == ["s1", "s2", "s3", "s4", "s5"]      # lexicographic; s5 label-only
    assert ds.n_songs == 4 and ds.n_extra_songs == 1 and ds.n_label_songs == 3
    assert ds.song_count.tolist() == [2, 3, 3, 2]       # train AND test listens (MR:60-62)
    assert [ds.train_names(i) for i in range(3)] == ["A", "B", "C"]
    assert ds.tr_len.tolist() == [3, 2, 2] and ds.te_len.tolist() == [2, 1]


def test_duplicates_counted_in_lengths_not_in_rows():
    K = kat()["dup"]
    ds = dataset_from_lines(K["train"], K["test"], K["labels"])
    assert ds.song_count.tolist() == [4, 3, 3, 3]       # s1: A,A,X,X ; s4: C,C,X
    assert ds.tr_len.tolist() == [4, 2, 3] and ds.te_len.tolist() == [3, 1]
    assert ds.tr_off.tolist() == [0, 3, 5, 7]           # rows stay sets


def test_matches_numpy_builder_on_synthetic(tmp_path):
    t = synth.config("small")
    a = t.dataset()
    paths = [str(tmp_path / n) for n in ("train.txt", "test.txt", "labels.txt")]
    a.write_tsv(*paths)
    b = Dataset.from_tsv(*paths)
    for f in ("n_train", "n_test", "n_songs", "n_label_songs", "n_extra_songs"):
        assert getattr(a, f) == getattr(b, f), f
    for f in ("tr_off", "tr_songs", "te_off", "te_songs", "song_count", "tr_len", "te_len", "lab_off", "lab_songs"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    assert [a.song_names(i) for i in range(a.n_songs)] == [b.song_names(i) for i in range(b.n_songs)]


@pytest.mark.parametrize("bad", ["u\ts", "u\ts\t1\t2", "", "u\t\t1\tx"])
def test_malformed_lines_are_parse_errors(tmp_path, bad):
    (tmp_path / "tr").write_text("a\tb\t1\n" + bad + "\n")
    (tmp_path / "te").write_text("x\tb\t1\n")
    with pytest.raises(_lib.EngineError) as ei:
        Dataset.from_tsv(str(tmp_path / "tr"), str(tmp_path / "te"), None)
    assert ei.value.code == _lib.MR_E_PARSE


def test_java_split_trailing_fields_and_crlf(tmp_path):
    # "u\ts\t3\t" -> Java split drops the trailing empty field -> 3 fields, OK
    (tmp_path / "tr").write_text("a\tb\t3\t\r\nc\tb\t1\n")
    (tmp_path / "te").write_text("x\tb\t1\r\n")
    ds = Dataset.from_tsv(str(tmp_path / "tr"), str(tmp_path / "te"), None)
    assert ds.n_train == 2 and ds.n_songs == 1 and ds.song_count.tolist() == [3]


def test_missing_file_and_overlapping_users(tmp_path):
    with pytest.raises(_lib.EngineError) as ei:
        Dataset.from_tsv(str(tmp_path / "nope"), str(tmp_path / "nope2"), None)
    assert ei.value.code == _lib.MR_E_IO
    (tmp_path / "tr").write_text("a\tb\t1\n")
    (tmp_path / "te").write_text("a\tc\t1\n")
    with pytest.raises(_lib.EngineError) as ei:
        Dataset.from_tsv(str(tmp_path / "tr"), str(tmp_path / "te"), None)
    assert ei.value.code == _lib.MR_E_INVALID


def test_subset_test_users_keeps_global_counts():
    ds = synth.config("small").dataset()
    sub = ds.subset_test_users(2, 5)
    assert sub.n_test == 3 and np.array_equal(sub.song_count, ds.song_count)
    assert np.array_equal(sub.te_songs, ds.te_songs[ds.te_off[2]:ds.te_off[5]])
    fp_full, _, _ = native.fp_model(ds, "ibm")
    fp_sub, _, _ = native.fp_model(sub, "ibm")
    assert np.array_equal(fp_full[2:5], fp_sub, equal_nan=True)


def test_synthetic_generator_shapes():
    for name, target in (("c1", 4798), ("c2", 16785)):
        ds = synth.config(name).dataset()
        assert abs(ds.n_songs - target) / target < 0.05
    a = synth.config("c2").dataset()
    b = synth.config("c2", n_test=30).dataset()
    # prefix-consistent: the first 10 test users and the train set are unchanged
    assert np.array_equal(a.tr_len, b.tr_len)
    assert np.array_equal(a.te_len, b.te_len[:10])


@pytest.mark.parametrize("threads", ["1", "3", "8"])
def test_parallel_chunks_identical(tmp_path, monkeypatch, threads):
    """The multi-threaded reader (chunks cut at line starts, per-thread
    interning merged afterwards) gives the single-thread corpus; parse errors
    report the first bad line of the file whichever chunk holds it."""
    t = synth.config("small")
    a = t.dataset()
    paths = [str(tmp_path / n) for n in ("train.txt", "test.txt", "labels.txt")]
    a.write_tsv(*paths)
    monkeypatch.setenv("MR_INGEST_MIN_CHUNK", "97")
    monkeypatch.setenv("MR_INGEST_THREADS", threads)
    b = Dataset.from_tsv(*paths)
    for f in ("tr_off", "tr_songs", "te_off", "te_songs", "song_count", "tr_len", "te_len", "lab_off", "lab_songs"):
        assert np.array_equal(getattr(a, f), getattr(b, f)), f
    lines = open(paths[0]).read().splitlines()
    lines[len(lines) // 2] = "broken"
    lines[len(lines) - 3] = "also\tbroken"
    with open(paths[0], "w") as f:
        f.write("\n".join(lines) + "\n")
    with pytest.raises(_lib.EngineError) as ei:
        Dataset.from_tsv(*paths)
    assert ei.value.code == _lib.MR_E_PARSE and f":{len(lines) // 2 + 1}:" in str(ei.value)


def test_bulk_names_errors_and_empty_names(tmp_path):
    """mr_corpus_names: every name in id order, each followed by a newline
    (empty names included); bad kind / short buffer are error codes."""
    import ctypes

    (tmp_path / "tr.txt").write_text("u1\ts2\t1\nu0\ts1\t1\n\ts1\t1\n")  # an empty user name (Java split keeps it)
    (tmp_path / "te.txt").write_text("t0\ts2\t1\n")
    ds = Dataset.from_tsv(str(tmp_path / "tr.txt"), str(tmp_path / "te.txt"))
    assert [ds.train_names(i) for i in range(ds.n_train)] == ["", "u0", "u1"]
    assert [ds.song_names(i) for i in range(ds.n_songs)] == ["s1", "s2"]
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.mr_corpus_from_tsv(os.fsencode(str(tmp_path / "tr.txt")), os.fsencode(str(tmp_path / "te.txt")),
                                    None, ctypes.byref(h)), "mr_corpus_from_tsv")
    try:
        need = ctypes.c_int64()
        assert L.mr_corpus_names(h, 1, None, 0, ctypes.byref(need)) == 0 and need.value == len("\nu0\nu1\n")
        small = ctypes.create_string_buffer(2)
        assert L.mr_corpus_names(h, 1, small, 2, ctypes.byref(need)) == _lib.MR_E_INVALID
        assert L.mr_corpus_names(h, 7, None, 0, ctypes.byref(need)) == _lib.MR_E_INVALID
    finally:
        L.mr_corpus_free(h)
